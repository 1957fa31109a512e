"""Aggregator function entry point without MongoDB.

Restates fedless/aggregator/aggregation.py:45-167 (default_aggregation_handler)
over the in-memory stores of fedlesscan_amd.store, and
fedless/controller/mocks/mock_aggregation.py:6-31 (MockAggregator, the
in-process caller of BASELINE config 1).  Steps, in the reference's order:

  1. strategy factory: PER_SESSION -> StallAwareAggregator(R, hp), else FedAvg  (:71-75)
  2. select_aggregation_candidates (round, or session with tolerance)         (:76-78)
  3. aggregate_online -> stream variant, else materialise the results          (:79-93)
  4. aggregate -> new parameters (HIP fold)                                    (:95-97)
  5. serialise with the configured serializer, save as round R+1              (:125-138)
  6. count (round or whole session) and optionally delete the results          (:141-153)
  7. AggregatorFunctionResult(new_round_id=R+1, num_clients=count, ...)        (:158-163)
SerializationError / store errors surface as AggregationError (:164-165).

Divergences (documented in DESIGN.md): global evaluation with Keras
(`test_data`, :100-123) is out of scope and raises; aggregation_hyper_params
=None is treated as the defaults (the reference dereferences it, App. C.6).
"""
from __future__ import annotations

import logging
from typing import Optional

from .aggregator import (
    AggregationError,
    FedAvgAggregator,
    StallAwareAggregator,
    StreamFedAvgAggregator,
    StreamStallAwareAggregator,
)
from .common.models import (
    AggregationHyperParams,
    AggregationStrategy,
    AggregatorFunctionParams,
    AggregatorFunctionResult,
    SerializedParameters,
    WeightsSerializerConfig,
)
from .common.serialization import SerializationError, WeightsSerializerBuilder
from .store import DocumentNotLoadedException, InMemoryClientResultStore, InMemoryParameterStore

logger = logging.getLogger(__name__)


def default_aggregation_handler(session_id: str, round_id: int, result_store: InMemoryClientResultStore,
                                parameter_store: InMemoryParameterStore, serializer: WeightsSerializerConfig,
                                test_data=None, delete_results_after_finish: bool = True,
                                aggregation_strategy: AggregationStrategy = AggregationStrategy.PER_ROUND,
                                aggregation_hyper_params: Optional[AggregationHyperParams] = None,
                                device=None, devices=None) -> AggregatorFunctionResult:
    """device / devices: the GPU, or several GPUs of this process (one column
    bucket each, fedlesscan_amd.multigpu), the strategy folds on."""
    hp = aggregation_hyper_params if aggregation_hyper_params is not None else AggregationHyperParams()
    per_session = aggregation_strategy == AggregationStrategy.PER_SESSION
    logger.info(f"Aggregator invoked for session {session_id} and round {round_id}")
    try:
        aggregator = (StallAwareAggregator(round_id, hp, device=device, devices=devices) if per_session
                      else FedAvgAggregator(device=device, devices=devices))
        feats, results = aggregator.select_aggregation_candidates(result_store, session_id, round_id)
        if hp.aggregate_online:
            aggregator = (StreamStallAwareAggregator(round_id, hp, device=device, devices=devices) if per_session
                          else StreamFedAvgAggregator(device=device, devices=devices))
        else:
            results = results if isinstance(results, list) else list(results)
        new_parameters, test_results = aggregator.aggregate(results, feats)

        if test_data:
            raise AggregationError("global evaluation (test_data) needs Keras and is out of scope")

        blob = WeightsSerializerBuilder.from_config(serializer).serialize(new_parameters)
        new_round_id = round_id + 1
        parameter_store.save(session_id=session_id, round_id=new_round_id,
                             params=SerializedParameters(blob=blob, serializer=serializer))
        if per_session:
            processed = result_store.count_results_for_session(session_id=session_id)
            if delete_results_after_finish:
                result_store.delete_results_for_session(session_id=session_id)
        else:
            processed = result_store.count_results_for_round(session_id=session_id, round_id=round_id)
            if delete_results_after_finish:
                result_store.delete_results_for_round(session_id=session_id, round_id=round_id)
        return AggregatorFunctionResult(new_round_id=new_round_id, num_clients=processed,
                                        test_results=test_results, global_test_results=None)
    except (SerializationError, DocumentNotLoadedException) as e:
        raise AggregationError(e) from e


class MockAggregator:
    """In-process aggregator (mock_aggregation.py:6-31) over the in-memory stores."""

    def __init__(self, params: AggregatorFunctionParams, result_store: InMemoryClientResultStore,
                 parameter_store: InMemoryParameterStore, delete_results_after_finish: bool = True, device=None,
                 devices=None):
        self.params = params
        self.devices = devices
        self.result_store = result_store
        self.parameter_store = parameter_store
        self.delete_results_after_finish = delete_results_after_finish
        self.device = device

    def run_aggregator(self) -> AggregatorFunctionResult:
        p = self.params
        return default_aggregation_handler(p.session_id, p.round_id, self.result_store, self.parameter_store,
                                           p.serializer, None, self.delete_results_after_finish,
                                           p.aggregation_strategy, p.aggregation_hyper_params, self.device,
                                           self.devices)
