"""fedlesscan_amd — MI355X-native FedAvg / FedLesScan parameter aggregation.

Drop-in for the reference's aggregation hot path (fedless/aggregator/*): the
strategy classes keep their signatures; the weighted fold runs in hand-written
gfx950 HIP kernels (libfedavg_hip.so, C-ABI in include/fedavg_hip.h) called
through ctypes.  See DESIGN.md.
"""
__version__ = "0.1.0"

from .aggregator import (  # noqa: F401,E402
    AggregationError,
    FedAvgAggregator,
    InsufficientClientResults,
    InvalidParameterShapeError,
    ParameterAggregator,
    StallAwareAggregator,
    StreamFedAvgAggregator,
    StreamStallAwareAggregator,
    UnknownCardinalityError,
)
