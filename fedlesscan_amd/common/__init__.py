"""Schemas and wire-format codecs on the aggregation path."""
