"""Wire/config schemas on the aggregation path (pydantic v2).

Mirrors the subset of fedless/common/models the hot path touches:
  Parameters                  models.py:22
  TestMetrics                 models.py:32-38
  NpzWeightsSerializerConfig  models.py:49-54
  BinaryStringFormat          models.py:57-59
  WeightsSerializerConfig     models.py:150-159
  SerializedParameters        models.py:165-170
  ClientResult                models.py:181-193
  AggregationStrategy / AggregationHyperParams / AggregatorFunctionResult
                              aggregation_models.py:14-41
"""
from __future__ import annotations

from enum import Enum
from typing import Dict, List, Literal, Optional, Union

import numpy as np
from pydantic import BaseModel, ConfigDict, Field

Parameters = List[np.ndarray]


class TestMetrics(BaseModel):
    __test__ = False  # not a pytest class
    cardinality: int
    metrics: Dict


class NpzWeightsSerializerConfig(BaseModel):
    type: Literal["npz"] = "npz"
    compressed: bool = False


class BinaryStringFormat(str, Enum):
    BASE64 = "base64"
    NONE = "none"


class WeightsSerializerConfig(BaseModel):
    type: str
    params: NpzWeightsSerializerConfig


class SerializedParameters(BaseModel):
    blob: Union[bytes, str]
    serializer: WeightsSerializerConfig
    string_format: BinaryStringFormat = BinaryStringFormat.NONE


class ClientResult(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)
    parameters: Optional[SerializedParameters] = None
    history: Optional[Dict] = None
    test_metrics: Optional[TestMetrics] = None
    cardinality: int
    privacy_guarantees: Optional[Dict] = None


class AggregationStrategy(str, Enum):
    PER_ROUND = "per_round"
    PER_SESSION = "per_session"


class AggregationHyperParams(BaseModel):
    tolerance: int = 0
    aggregate_online: bool = False
    test_batch_size: int = 10


class AggregatorFunctionResult(BaseModel):
    new_round_id: int
    num_clients: int
    test_results: Optional[List[TestMetrics]] = None
    global_test_results: Optional[TestMetrics] = None


class AggregatorFunctionParams(BaseModel):
    """aggregation_models.py:25-34.  `database` (the MongoDB connection) is
    accepted so the reference controller's requests parse, but results and
    parameters come from the in-memory stores; `test_data` (Keras global
    evaluation) is out of scope and the handler refuses a non-null one."""
    session_id: str
    round_id: int
    database: Optional[Dict] = None
    test_data: Optional[Dict] = None
    serializer: WeightsSerializerConfig = Field(
        default_factory=lambda: WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig()))
    aggregation_hyper_params: AggregationHyperParams = Field(default_factory=AggregationHyperParams)
    aggregation_strategy: AggregationStrategy = AggregationStrategy.PER_ROUND
