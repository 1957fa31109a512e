"""BSON documents as the reference persists client results and global models.

The reference keeps every ClientResult and every SerializedParameters as one
BSON document in GridFS:

  ClientResultDao.save   client_daos.py:73   _gridfs.put(bson.encode(result.dict()))
  ClientResultDao load   client_daos.py:142  ClientResult.parse_obj(bson.decode(file.read()))
  ParameterDao.save      client_daos.py:369  _gridfs.put(bson.encode(params.dict()))
  ParameterDao.load      client_daos.py:397  SerializedParameters.parse_obj(bson.decode(...))

`bson` there is pymongo's codec (pymongo~=3.11.3, requirements/requirements.txt:8;
bsonspec.org 1.1).  This module restates the part of it those documents use:

  decode(data, zero_copy)   element table from one native fa_bson_walk call
                            (C++, bounds-checked); binary subtype 0 comes back as a
                            memoryview into `data` when zero_copy, so a 40 MB NPZ
                            blob is never copied on its way to pinned staging
  encode(doc)               byte-identical to bson.encode for dict / list /
                            tuple / str / str-Enum / bytes / bool / int / float
                            / None / datetime (tests/test_bson.py checks against
                            pymongo where it is importable)
  client_result_from_bson   ClientResult.parse_obj(bson.decode(...)) with the
                            blob left as a view
  parameters_from_bson      SerializedParameters.parse_obj(bson.decode(...))

Decoding follows pymongo's default CodecOptions: documents are dicts, int32 is int,
int64 is Int64 (an int subclass), datetimes are naive UTC, binary subtype 0 is bytes.  Other
binary subtypes come back as `Binary`.  Decimal128, regex, code and DBPointer
values raise InvalidBSON: no persisted FedLesScan document holds them.
"""
from __future__ import annotations

import datetime as _dt
import struct
import threading
from enum import Enum
from typing import Any, Dict, Tuple

import numpy as np

from . import _lib
from .common.models import ClientResult, SerializedParameters


class InvalidBSON(ValueError):
    """Malformed or unsupported BSON (bson.errors.InvalidBSON in the reference)."""


class InvalidDocument(ValueError):
    """A value encode() cannot represent (bson.errors.InvalidDocument)."""


class Binary(bytes):
    """Binary payload with a non-default subtype (bson.binary.Binary)."""

    def __new__(cls, data, subtype: int = 0):
        o = super().__new__(cls, data)
        o.subtype = subtype
        return o

    def __eq__(self, other):
        return isinstance(other, Binary) and other.subtype == self.subtype and bytes(self) == bytes(other)

    def __hash__(self):
        return hash((bytes(self), self.subtype))


class Int64(int):
    """A BSON int64 (type 0x12) kept as int64 on re-encode (bson.int64.Int64)."""


class ObjectId(bytes):
    """12-byte ObjectId (bson.objectid.ObjectId); str() is its hex form."""

    def __str__(self):
        return self.hex()


_EPOCH = _dt.datetime(1970, 1, 1)
_I32, _I64, _F64 = struct.Struct("<i"), struct.Struct("<q"), struct.Struct("<d")
_MAX_ELEMS = 64
FA_BSON_MALFORMED, FA_BSON_UNSUPPORTED = -1, -2  # include/fedavg_hip.h


class _Scratch:
    """Output arrays for fa_bson_walk, one set per thread, grown on demand."""

    def __init__(self, cap: int = _MAX_ELEMS):
        self.grow(cap)

    def grow(self, cap: int):
        self.cap = cap
        self.ty = np.empty(cap, np.uint8)
        self.pa = np.empty(cap, np.int32)
        self.no = np.empty(cap, np.int64)
        self.nl = np.empty(cap, np.int32)
        self.vo = np.empty(cap, np.int64)
        self.vl = np.empty(cap, np.int64)
        self.st = np.empty(cap, np.uint8)
        self.ptrs = [a.ctypes.data for a in (self.ty, self.pa, self.no, self.nl, self.vo, self.vl, self.st)]


_tls = threading.local()


def _walk(buf: memoryview, base: int):
    """Flat pre-order element table of the whole document (one native call)."""
    sc = getattr(_tls, "scratch", None)
    if sc is None:
        sc = _tls.scratch = _Scratch()
    fn = _lib.load().fa_bson_walk
    while True:
        n = fn(base, len(buf), 0, *sc.ptrs, sc.cap)
        if n == FA_BSON_UNSUPPORTED:
            raise InvalidBSON("unsupported BSON element type")
        if n < 0:
            raise InvalidBSON("malformed BSON document")
        if n <= sc.cap:
            return (sc.ty[:n].tolist(), sc.pa[:n].tolist(), sc.no[:n].tolist(), sc.nl[:n].tolist(),
                    sc.vo[:n].tolist(), sc.vl[:n].tolist(), sc.st[:n].tolist())
        sc.grow(int(n))


def _scalar(buf: memoryview, t: int, vo: int, vl: int, st: int, zero_copy: bool):
    if t == 0x01:
        return _F64.unpack_from(buf, vo)[0]
    if t == 0x02:
        try:
            return str(buf[vo:vo + vl], "utf-8")
        except UnicodeDecodeError as e:
            raise InvalidBSON(f"invalid UTF-8 string: {e}") from e
    if t == 0x05:
        raw = buf[vo:vo + vl]
        if st == 0:
            return raw if zero_copy else raw.tobytes()
        return Binary(raw.tobytes(), st)
    if t in (0x06, 0x0A):
        return None
    if t == 0x07:
        return ObjectId(buf[vo:vo + 12].tobytes())
    if t == 0x08:
        return buf[vo] == 1
    if t == 0x09:
        ms = _I64.unpack_from(buf, vo)[0]
        try:
            return _EPOCH + _dt.timedelta(milliseconds=ms)
        except OverflowError as e:
            raise InvalidBSON(f"datetime out of range: {ms} ms") from e
    if t == 0x10:
        return _I32.unpack_from(buf, vo)[0]
    if t == 0x11:
        inc, ts = struct.unpack_from("<II", buf, vo)
        return (ts, inc)
    if t == 0x12:
        return Int64(_I64.unpack_from(buf, vo)[0])
    raise InvalidBSON(f"BSON type 0x{t:02x} is not used by persisted FedLesScan documents")


def decode(data, zero_copy: bool = False) -> Dict[str, Any]:
    """bson.decode(data) for one whole document (trailing bytes are an error)."""
    buf = memoryview(data).cast("B")
    if len(buf) < 5:
        raise InvalidBSON("not enough data for a BSON document")
    if _I32.unpack_from(buf, 0)[0] != len(buf):
        raise InvalidBSON("BSON document length does not match the data")
    arr = np.frombuffer(buf, dtype=np.uint8)  # keeps the address valid for the walk
    ty, pa, no, nl, vo, vl, st = _walk(buf, arr.ctypes.data)
    root: Dict[str, Any] = {}
    containers: Dict[int, Any] = {-1: root}
    for k in range(len(ty)):
        t = ty[k]
        if t == 0x03:
            v = containers[k] = {}
        elif t == 0x04:
            v = containers[k] = []
        else:
            v = _scalar(buf, t, vo[k], vl[k], st[k], zero_copy)
        parent = containers[pa[k]]
        if isinstance(parent, list):
            parent.append(v)
        else:
            try:
                parent[str(buf[no[k]:no[k] + nl[k]], "utf-8")] = v
            except UnicodeDecodeError as e:
                raise InvalidBSON(f"invalid UTF-8 key: {e}") from e
    return root


# ---------------------------------------------------------------------------
# encode
# ---------------------------------------------------------------------------
def _cstring(name: str) -> bytes:
    b = name.encode("utf-8")
    if b"\x00" in b:
        raise InvalidDocument(f"BSON keys must not contain a NUL character: {name!r}")
    return b + b"\x00"


def _encode_value(parts: list, name: bytes, v) -> int:
    """Append one element's chunks to `parts`; return its byte count."""
    if isinstance(v, Enum) and isinstance(v, str):
        v = v.value
    head = 1 + len(name)
    if v is None:
        parts += (b"\x0a", name)
        return head
    if isinstance(v, bool):
        parts += (b"\x08", name, b"\x01" if v else b"\x00")
        return head + 1
    if isinstance(v, int):
        if -(1 << 31) <= v < (1 << 31) and not isinstance(v, Int64):
            parts += (b"\x10", name, _I32.pack(v))
            return head + 4
        if -(1 << 63) <= v < (1 << 63):
            parts += (b"\x12", name, _I64.pack(v))
            return head + 8
        raise OverflowError("BSON can only handle up to 8-byte ints")
    if isinstance(v, float):
        parts += (b"\x01", name, _F64.pack(v))
        return head + 8
    if isinstance(v, str):
        b = v.encode("utf-8")
        parts += (b"\x02", name, _I32.pack(len(b) + 1), b, b"\x00")
        return head + 5 + len(b)
    if isinstance(v, (bytes, memoryview)):
        n = memoryview(v).nbytes
        parts += (b"\x05", name, _I32.pack(n), bytes((getattr(v, "subtype", 0),)), v)
        return head + 5 + n
    if isinstance(v, dict):
        parts += (b"\x03", name)
        return head + _encode_doc(parts, v.items())
    if isinstance(v, (list, tuple)):
        parts += (b"\x04", name)
        return head + _encode_doc(parts, ((str(i), x) for i, x in enumerate(v)))
    if isinstance(v, _dt.datetime):
        if v.tzinfo is not None:
            v = v.astimezone(_dt.timezone.utc).replace(tzinfo=None)
        delta = v - _EPOCH
        ms = (delta.days * 86400 + delta.seconds) * 1000 + delta.microseconds // 1000
        parts += (b"\x09", name, _I64.pack(ms))
        return head + 8
    raise InvalidDocument(f"cannot encode object: {v!r}, of type: {type(v)}")


def _encode_doc(parts: list, items) -> int:
    at = len(parts)
    parts.append(b"")  # int32 length, patched below
    n = 5
    for k, v in items:
        if not isinstance(k, str):
            raise InvalidDocument(f"documents must have only string keys, key was {k!r}")
        n += _encode_value(parts, _cstring(k), v)
    parts.append(b"\x00")
    parts[at] = _I32.pack(n)
    return n


def encode(doc: Dict[str, Any]) -> bytes:
    """bson.encode(doc).  Chunks are gathered and joined once, so every payload
    (the NPZ blob) is copied exactly once into the output."""
    if not isinstance(doc, dict):
        raise TypeError(f"encode() takes a dict, not {type(doc)}")
    parts: list = []
    _encode_doc(parts, doc.items())
    return b"".join(parts)


def encode_into(doc: Dict[str, Any], alloc) -> memoryview:
    """encode(doc) written into alloc(size), a writable byte buffer of exactly
    `size` bytes (e.g. pinned.pinned_bytes); same bytes, same single copy."""
    if not isinstance(doc, dict):
        raise TypeError(f"encode_into() takes a dict, not {type(doc)}")
    parts: list = []
    size = _encode_doc(parts, doc.items())
    out = memoryview(alloc(size)).cast("B")
    if len(out) != size:
        raise ValueError(f"alloc returned {len(out)} bytes, expected {size}")
    pos = 0
    for part in parts:
        n = memoryview(part).nbytes
        out[pos:pos + n] = memoryview(part).cast("B")
        pos += n
    return out


# ---------------------------------------------------------------------------
# the two persisted document kinds
# ---------------------------------------------------------------------------
def _take_blob(d: dict) -> Tuple[dict, Any]:
    params = d.get("parameters") if "parameters" in d else d
    if isinstance(params, dict) and isinstance(params.get("blob"), memoryview):
        blob = params["blob"]
        params["blob"] = b""
        return d, blob
    return d, None


def client_result_from_bson(data, zero_copy: bool = True) -> ClientResult:
    """ClientResult.parse_obj(bson.decode(data)) (client_daos.py:142).  With
    zero_copy the NPZ blob stays a read-only view into `data` (assigned after
    validation, so pydantic never copies it)."""
    d, blob = _take_blob(decode(data, zero_copy=zero_copy))
    cr = ClientResult.model_validate(d)
    if blob is not None and cr.parameters is not None:
        cr.parameters.blob = blob
    return cr


def parameters_from_bson(data, zero_copy: bool = False) -> SerializedParameters:
    """SerializedParameters.parse_obj(bson.decode(data)) (client_daos.py:397)."""
    d, blob = _take_blob(decode(data, zero_copy=zero_copy))
    sp = SerializedParameters.model_validate(d)
    if blob is not None:
        sp.blob = blob
    return sp
