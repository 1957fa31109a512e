"""NPZ weights (de)serialisation on the aggregation path.

Mirrors fedless/common/serialization.py:
  deserialize_parameters     :80-93
  Base64StringConverter      :140-171
  NpzWeightsSerializer       :280-306  (np.savez / np.load of an in-memory zip;
                                        allow_pickle stays False)
  WeightsSerializerBuilder   :309-324
ValueError / IOError during (de)serialisation surface as SerializationError
(:56-73, wrap_exceptions_as_serialization_error).
"""
from __future__ import annotations

import base64
import binascii
import io
from typing import List

import numpy as np

from .models import BinaryStringFormat, NpzWeightsSerializerConfig, SerializedParameters, WeightsSerializerConfig


class SerializationError(Exception):
    pass


class Base64StringConverter:
    @staticmethod
    def get_format() -> BinaryStringFormat:
        return BinaryStringFormat.BASE64

    @staticmethod
    def to_str(obj: bytes) -> str:
        return base64.b64encode(obj).decode("ascii")

    @staticmethod
    def from_str(rep: str) -> bytes:
        try:
            return base64.b64decode(rep)
        except binascii.Error:
            raise ValueError("Given string is not in base64 or incorrectly padded")


class NpzWeightsSerializer:
    def __init__(self, compressed: bool = False):
        self.compressed = compressed

    def get_config(self) -> WeightsSerializerConfig:
        p = NpzWeightsSerializerConfig(compressed=self.compressed)
        return WeightsSerializerConfig(type=p.type, params=p)

    def serialize(self, weights: List[np.ndarray]) -> bytes:
        # not wrapped: only deserialize carries wrap_exceptions_as_serialization_error
        # (serialization.py:292-306), so e.g. serialize(None) raises TypeError
        if not self.compressed:
            # byte-identical np.savez with native checksums (fedlesscan_amd/npz.py)
            from ..npz import write_npz
            b = write_npz(weights)
            if b is not None:
                return b
        with io.BytesIO() as f:
            (np.savez_compressed if self.compressed else np.savez)(f, *weights)
            return f.getvalue()

    def deserialize(self, blob: bytes) -> List[np.ndarray]:
        try:
            with io.BytesIO(blob) as f:
                with np.load(f, allow_pickle=False) as npz:
                    return [npz[k] for k in npz.files]
        except MemoryError:
            raise
        except Exception as e:  # np.load raises ValueError / OSError / BadZipFile
            raise SerializationError(e) from e


class WeightsSerializerBuilder:
    @staticmethod
    def from_config(config: WeightsSerializerConfig) -> NpzWeightsSerializer:
        if config.type == "npz":
            return NpzWeightsSerializer(compressed=config.params.compressed)
        raise NotImplementedError(f"Serializer of type {config.type} does not exist")


def deserialize_parameters(serialized: SerializedParameters, zero_copy: bool = False) -> List[np.ndarray]:
    """serialization.py:80-93.  zero_copy=True returns read-only views into the
    blob for uncompressed NPZ (fedlesscan_amd.npz) -- same values, no copy."""
    serializer = WeightsSerializerBuilder.from_config(serialized.serializer)
    if serialized.string_format == BinaryStringFormat.BASE64:
        try:
            blob = Base64StringConverter.from_str(serialized.blob)
        except ValueError as e:
            raise SerializationError(e) from e
    elif serialized.string_format == BinaryStringFormat.NONE:
        blob = serialized.blob
    else:
        raise SerializationError(f"Binary string format {serialized.string_format} not known")
    if zero_copy and not serializer.compressed:
        from ..npz import read_layers
        try:
            return read_layers(blob)
        except MemoryError:
            raise
        except Exception as e:
            raise SerializationError(e) from e
    return serializer.deserialize(blob)
