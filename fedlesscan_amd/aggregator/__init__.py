"""Drop-in aggregation strategies (mirror of fedless.aggregator)."""
from .exceptions import (  # noqa: F401
    AggregationError,
    InsufficientClientResults,
    InvalidParameterShapeError,
    UnknownCardinalityError,
)
from .parameter_aggregator import ParameterAggregator  # noqa: F401
from .fed_avg_aggregator import FedAvgAggregator, StreamFedAvgAggregator  # noqa: F401
from .stall_aware_aggregation import StallAwareAggregator, StreamStallAwareAggregator  # noqa: F401
