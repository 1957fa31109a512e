"""Strategy plugin API (mirrors fedless/aggregator/parameter_aggregator.py:11-25)."""
import abc
from typing import Iterator, List, Optional, Tuple

from ..common.models import ClientResult, Parameters, TestMetrics


class ParameterAggregator(abc.ABC):
    """Select the client results of a round, then aggregate them."""

    @abc.abstractmethod
    def select_aggregation_candidates(self, **kwargs) -> Iterator:
        pass

    @abc.abstractmethod
    def aggregate(self, client_results: Iterator[ClientResult], client_feats: List[dict]
                  ) -> Tuple[Parameters, Optional[List[TestMetrics]]]:
        pass
