"""FedAvg strategies on the MI355X engine.

Drop-in for fedless/aggregator/fed_avg_aggregator.py:
  FedAvgAggregator._aggregate                  :24-42   -> engine.aggregate_layers (HIP fold)
  FedAvgAggregator.select_aggregation_candidates :44-55
  FedAvgAggregator.aggregate                   :57-92
  StreamFedAvgAggregator.chunks / .aggregate   :95-153

Same constructor signatures, argument meaning, return types and exceptions.
`select_aggregation_candidates(mongo_client, session_id, round_id)` takes a
result store with the ClientResultDao query methods (the reference's DAO, or
fedlesscan_amd.store.InMemoryClientResultStore), or a pymongo client, which
it wraps into the reference's ClientResultDao as the reference does
(parameter_aggregator.result_store).
"""
from __future__ import annotations

import logging
from typing import Iterable, Iterator, List, Optional, Tuple

import numpy as np

from .. import engine
from ..common.models import ClientResult, Parameters, TestMetrics
from ..common.serialization import deserialize_parameters
from .exceptions import InsufficientClientResults, UnknownCardinalityError
from .parameter_aggregator import ParameterAggregator, result_store

logger = logging.getLogger(__name__)

# tf.data.UNKNOWN_CARDINALITY / tf.data.INFINITE_CARDINALITY
UNKNOWN_CARDINALITY = -2
INFINITE_CARDINALITY = -1


def resolve_cardinality(cardinality, default_cardinality):
    """fed_avg_aggregator.py:71-82.  Note the reference's `if not default`:
    a default of 0 / 0.0 counts as "no default" (SURVEY App. C.8)."""
    if cardinality in (UNKNOWN_CARDINALITY, INFINITE_CARDINALITY):
        if not default_cardinality:
            raise UnknownCardinalityError("Cardinality for client result invalid. ")
        return default_cardinality
    return cardinality


def decode_result(result: ClientResult, default_cardinality):
    """Deserialize one ClientResult and release its blob (`del client_result.parameters`)."""
    params = deserialize_parameters(result.parameters, zero_copy=True)
    result.parameters = None  # the reference's `del client_result.parameters`
    return params, resolve_cardinality(result.cardinality, default_cardinality), result.test_metrics


def decode_results(results: Iterable[ClientResult], default_cardinality):
    params, cards, metrics = [], [], []
    for r in results:
        p, c, m = decode_result(r, default_cardinality)
        params.append(p)
        cards.append(c)
        if m:
            metrics.append(m)
    return params, cards, metrics


def decoded_rows(results: Iterable[ClientResult], default_cardinality, metrics: list):
    """Lazy decode_results: yields (layers, cardinality), collects test metrics."""
    for r in results:
        p, c, m = decode_result(r, default_cardinality)
        if m:
            metrics.append(m)
        yield p, c


def chunked(items: Iterable, n: int) -> Iterator[list]:
    """Full chunks of n, then the remainder (fed_avg_aggregator.py:99-109)."""
    buf: list = []
    for el in items:
        buf.append(el)
        if len(buf) == n:
            yield buf
            buf = []
    if buf:
        yield buf


class FedAvgAggregator(ParameterAggregator):
    """Cardinality-weighted FedAvg; the fold runs in libfedavg_hip.so.

    device:  the GPU to fold on (default: the current one).
    devices: several GPUs of this process (a list of ints / torch.device, or
             "all"): the model's columns are split into one bucket per GPU,
             each GPU ingests and folds its own bucket (multigpu.py), and the
             model is reassembled on the host; bit-identical to one GPU."""

    def __init__(self, device=None, devices=None):
        self.device = device
        self.devices = devices

    def _aggregate(self, parameters: List[List[np.ndarray]], weights: List[float]) -> List[np.ndarray]:
        return engine.aggregate_layers(parameters, weights, None, device=self.device, devices=self.devices)

    def select_aggregation_candidates(self, mongo_client, session_id, round_id):
        """fed_avg_aggregator.py:44-55; mongo_client: a result store or a
        MongoClient (parameter_aggregator.result_store)."""
        store = result_store(mongo_client)
        dicts, candidates = store.load_results_for_round(session_id=session_id, round_id=round_id)
        # The reference tests `if not round_candidates` (:51-54), and round_candidates
        # is the generator _retrieve_result_files returns (client_daos.py:125,161):
        # always truthy, so InsufficientClientResults is never raised here.  An empty
        # round aggregates to [] and is saved as round R+1 with num_clients=0.
        if not candidates:
            raise InsufficientClientResults(
                f"Found no client results for session {session_id} and round {round_id}")
        return dicts, candidates

    def aggregate(self, client_results: Iterator[ClientResult], client_feats: Optional[List[dict]] = None,
                  default_cardinality: Optional[float] = None) -> Tuple[Parameters, Optional[List[TestMetrics]]]:
        if type(self)._aggregate is not FedAvgAggregator._aggregate:
            # a subclass's own _aggregate gets the decoded lists, as in the reference
            params, cards, metrics = decode_results(client_results, default_cardinality)
            return self._aggregate(params, cards), (metrics or None)
        metrics: list = []
        n = len(client_results) if hasattr(client_results, "__len__") else 0
        out = engine.aggregate_decoded(decoded_rows(client_results, default_cardinality, metrics),
                                       None, device=self.device, devices=self.devices, expected_rows=n)
        return out, (metrics or None)


class StreamFedAvgAggregator(FedAvgAggregator):
    """Online FedAvg over chunks: g <- FedAvg([g, *chunk], [W, *n_chunk]).

    Reproduces the reference's running re-weighting exactly (it is not
    bit-equal to batch FedAvg)."""

    def __init__(self, chunk_size: int = 25, device=None, devices=None):
        super().__init__(device, devices)
        self.chunk_size = chunk_size

    def chunks(self, iterator: Iterator, n) -> Iterator[List]:
        return chunked(iterator, n)

    def aggregate(self, client_results: Iterator[ClientResult], client_feats: Optional[List[dict]] = None,
                  default_cardinality: Optional[float] = None) -> Tuple[Parameters, Optional[List[TestMetrics]]]:
        g, w_seen, metrics = None, 0, []
        for chunk in self.chunks(client_results, self.chunk_size):
            params, cards, m = decode_results(chunk, default_cardinality)
            metrics.extend(m)
            if g is None:
                g = self._aggregate(params, cards)
            else:
                g = self._aggregate([g, *params], [w_seen, *cards])
            w_seen += sum(cards)
        return g, (metrics or None)
