"""FedLesScan staleness-aware strategies on the MI355X engine.

Drop-in for fedless/aggregator/stall_aware_aggregation.py:
  StallAwareAggregator.__init__                    :25-32
  StallAwareAggregator._score_clients              :34-40   s_i = (r_i + 1) / (R + 1)
  StallAwareAggregator._aggregate                  :42-67   -> engine.aggregate_layers(scores=s)
  StallAwareAggregator.select_aggregation_candidates :69-80 (round_id >= R - tolerance)
  StallAwareAggregator.aggregate                   :82-117
  StreamStallAwareAggregator                       :120-187

Reproduced as the reference computes it: each term is (x * n_i) * s_i and
the divisor is sum(n_i), not sum(n_i * s_i); the stream
variant re-scores client_feats from index 0 for every chunk (App. C.2).
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Tuple

import numpy as np

from .. import engine
from ..common.models import AggregationHyperParams, ClientResult, Parameters, TestMetrics
from .exceptions import InsufficientClientResults
from .fed_avg_aggregator import chunked, decode_results, decoded_rows
from .parameter_aggregator import ParameterAggregator, result_store


class StallAwareAggregator(ParameterAggregator):
    def __init__(self, current_round, aggregation_hyper_params: Optional[AggregationHyperParams], device=None,
                 devices=None):
        self.current_round = current_round
        self.tolerance = aggregation_hyper_params.tolerance if aggregation_hyper_params is not None else 0
        self.device = device
        self.devices = devices  # several GPUs, one column bucket each (see FedAvgAggregator)
        super().__init__()

    def _score_clients(self, client_result: List[dict]) -> List[float]:
        denom = self.current_round + 1
        return [(d["round_id"] + 1) / denom for d in client_result]

    def _aggregate(self, client_feats: List[dict], parameters: List[List[np.ndarray]],
                   weights: List[float]) -> List[np.ndarray]:
        return engine.aggregate_layers(parameters, weights, self._score_clients(client_feats),
                                       device=self.device, devices=self.devices)

    def select_aggregation_candidates(self, mongo_client, session_id, round_id):
        """stall_aware_aggregation.py:69-80; mongo_client: a result store or a
        MongoClient (parameter_aggregator.result_store)."""
        store = result_store(mongo_client)
        dicts, candidates = store.load_results_for_session(session_id=session_id, round_id=round_id,
                                                           tolerance=self.tolerance)
        # always-truthy generator, as in the reference (:76-79): see FedAvgAggregator
        if not candidates:
            raise InsufficientClientResults(
                f"Found no client results for session {session_id} and round {round_id}")
        return dicts, candidates

    def aggregate(self, client_results: Iterator[ClientResult], client_feats: List[dict],
                  default_cardinality: Optional[float] = None) -> Tuple[Parameters, Optional[List[TestMetrics]]]:
        if type(self)._aggregate is not StallAwareAggregator._aggregate:
            params, cards, metrics = decode_results(client_results, default_cardinality)
            return self._aggregate(client_feats, params, cards), (metrics or None)
        metrics: list = []
        n = len(client_results) if hasattr(client_results, "__len__") else 0
        out = engine.aggregate_decoded(decoded_rows(client_results, default_cardinality, metrics),
                                       self._score_clients(client_feats), device=self.device,
                                       devices=self.devices, expected_rows=n)
        return out, (metrics or None)


class StreamStallAwareAggregator(StallAwareAggregator):
    def __init__(self, current_round: int, aggregation_hyper_params: Optional[AggregationHyperParams],
                 chunk_size: int = 25, device=None, devices=None):
        super().__init__(current_round, aggregation_hyper_params, device, devices)
        self.chunk_size = chunk_size

    def chunks(self, iterator: Iterator, n) -> Iterator[List]:
        return chunked(iterator, n)

    def aggregate(self, client_results: Iterator[ClientResult], client_feats: List[dict],
                  default_cardinality: Optional[float] = None) -> Tuple[Parameters, Optional[List[TestMetrics]]]:
        g, w_seen, metrics = None, 0, []
        for chunk in self.chunks(client_results, self.chunk_size):
            params, cards, m = decode_results(chunk, default_cardinality)
            metrics.extend(m)
            rows = params if g is None else [g, *params]
            weights = cards if g is None else [w_seen, *cards]
            g = self._aggregate(client_feats, rows, weights)
            w_seen += sum(cards)
        return g, (metrics or None)
