"""Error taxonomy of the aggregation path (mirrors fedless/aggregator/exceptions.py:1-14).

The C-ABI status codes map onto these classes in fedlesscan_amd._lib.
"""


class AggregationError(Exception):
    pass


class InsufficientClientResults(AggregationError):
    pass


class UnknownCardinalityError(AggregationError):
    pass


class InvalidParameterShapeError(AggregationError):
    """Raised for mismatched client layer shapes / dtypes.

    The reference defines this class but never raises it:
    numpy silently broadcasts compatible shapes or raises ValueError.  The
    engine rejects any shape mismatch explicitly -- a documented divergence.
    """
