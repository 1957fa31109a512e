"""Aggregator settings from an experiment config (the hot path's config inputs).

Restates only what reaches the aggregation path:
  AggregationFunctionConfig.hyperparams -> AggregationHyperParams
                                            (controller/models.py:25-28, aggregation_models.py:19-22)
  strategy name -> AggregationStrategy      (strategy_selector.py:12-36: "fedlesscan" -> PER_SESSION,
                                             "fedavg"/"fedprox" -> PER_ROUND, unknown -> fedlesscan)
YAML is read with yaml.safe_load; function endpoints, credentials and client
settings in the same file are ignored (out of scope).
"""
from __future__ import annotations

from typing import Tuple, Union

from .common.models import AggregationHyperParams, AggregationStrategy

_STRATEGIES = {"fedlesscan": AggregationStrategy.PER_SESSION, "fedavg": AggregationStrategy.PER_ROUND,
               "fedprox": AggregationStrategy.PER_ROUND}


def strategy_for(name: str) -> AggregationStrategy:
    """select_strategy's mapping, including its default to fedlesscan."""
    return _STRATEGIES.get(name, AggregationStrategy.PER_SESSION)


def aggregator_settings(config: Union[str, dict], strategy: str = "fedlesscan"
                        ) -> Tuple[AggregationStrategy, AggregationHyperParams]:
    if isinstance(config, str):
        import yaml
        with open(config) as f:
            config = yaml.safe_load(f)
    hp = ((config or {}).get("aggregator") or {}).get("hyperparams") or {}
    return strategy_for(strategy), AggregationHyperParams(**hp)
