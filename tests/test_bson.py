"""BSON documents as the reference persists them (client_daos.py:73, 142, 369,
397): fedlesscan_amd.bsondoc (native fa_bson_elements walk + Python values)
against pymongo's codec, the reference's own dependency (pymongo~=3.11.3,
requirements/requirements.txt:8; pymongo 4.x is what this image has -- the
BSON wire format is the same bsonspec 1.1).  pymongo is test infrastructure
here only: the product never imports it."""
import datetime
import random

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from fedlesscan_amd import bsondoc as B
from fedlesscan_amd.common.models import (BinaryStringFormat, ClientResult, NpzWeightsSerializerConfig,
                                          SerializedParameters, TestMetrics, WeightsSerializerConfig)
from fedlesscan_amd.common.serialization import Base64StringConverter, NpzWeightsSerializer

bson = pytest.importorskip("bson")

CFG = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())


def _result(i=0, b64=False, metrics=True, history=True):
    layers = [np.arange(12, dtype=np.float32).reshape(3, 4) * (i + 1), np.full(5, -i, np.float32)]
    raw = NpzWeightsSerializer().serialize(layers)
    sp = (SerializedParameters(blob=Base64StringConverter.to_str(raw), serializer=CFG,
                               string_format=BinaryStringFormat.BASE64) if b64
          else SerializedParameters(blob=raw, serializer=CFG))
    return ClientResult(parameters=sp, cardinality=100 + i,
                        history={"loss": [0.5, 0.25 * i], "accuracy": [0.75, 0.875]} if history else None,
                        test_metrics=TestMetrics(cardinality=10, metrics={"loss": 0.125, "accuracy": 0.5})
                        if metrics else None), layers


def _same(a, b):
    """Deep equality; memoryview == bytes compares contents."""
    if isinstance(a, dict):
        return isinstance(b, dict) and list(a) == list(b) and all(_same(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return isinstance(b, list) and len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, float) and a != a:
        return isinstance(b, float) and b != b
    if isinstance(a, bool) or isinstance(b, bool):
        return type(a) is type(b) and a == b
    if isinstance(a, B.Binary):
        return isinstance(b, bytes) and bytes(a) == bytes(b) and a.subtype == getattr(b, "subtype", 0)
    if isinstance(a, B.ObjectId):
        return isinstance(b, bson.ObjectId) and bytes(a) == b.binary
    if isinstance(a, tuple):  # Timestamp (time, inc)
        return isinstance(b, bson.Timestamp) and a == (b.time, b.inc)
    return a == b


# the value types a persisted ClientResult / SerializedParameters can hold
scalars = st.one_of(st.none(), st.booleans(), st.integers(-(1 << 63), (1 << 63) - 1),
                    st.floats(allow_nan=True), st.text(max_size=20), st.binary(max_size=40),
                    st.datetimes(min_value=datetime.datetime(1, 1, 1), max_value=datetime.datetime(9999, 12, 31))
                    .map(lambda d: d.replace(microsecond=d.microsecond // 1000 * 1000)))
keys = st.text(max_size=8).filter(lambda k: "\x00" not in k)
values = st.recursive(scalars, lambda ch: st.one_of(st.lists(ch, max_size=5),
                                                    st.dictionaries(keys, ch, max_size=5)), max_leaves=20)
docs = st.dictionaries(keys, values, max_size=8)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(d=docs)
def test_encode_decode_match_pymongo(d):
    ref = bson.encode(d)
    assert B.encode(d) == ref
    got = B.decode(ref)
    assert _same(got, bson.decode(ref))
    assert _same(B.decode(ref, zero_copy=True), got)


@pytest.mark.parametrize("b64", [False, True])
def test_client_result_document(b64):
    cr, layers = _result(3, b64=b64)
    data = B.encode(cr.model_dump())
    # the reference's bytes: pymongo over the same dict (pydantic v1 .dict() == v2 model_dump here)
    assert data == bson.encode(cr.model_dump())
    back = B.client_result_from_bson(data)
    ref = ClientResult.model_validate(bson.decode(data))
    assert back.cardinality == ref.cardinality == 103
    assert back.history == ref.history and back.test_metrics == ref.test_metrics
    assert back.parameters.string_format == ref.parameters.string_format
    assert back.parameters.serializer == ref.parameters.serializer
    if b64:
        assert back.parameters.blob == ref.parameters.blob and isinstance(back.parameters.blob, str)
    else:
        assert bytes(back.parameters.blob) == ref.parameters.blob
    if not b64:
        # zero copy: the blob is a view into the document bytes
        v = back.parameters.blob
        assert isinstance(v, memoryview)
        base = np.frombuffer(data, np.uint8).ctypes.data
        assert base <= np.frombuffer(v, np.uint8).ctypes.data < base + len(data)
    from fedlesscan_amd.common.serialization import deserialize_parameters
    for x, y in zip(deserialize_parameters(back.parameters, zero_copy=True), layers):
        assert np.array_equal(x, y) and x.dtype == y.dtype


def test_parameters_document():
    raw = NpzWeightsSerializer().serialize([np.ones(7, np.float32)])
    sp = SerializedParameters(blob=raw, serializer=CFG)
    data = B.encode(sp.model_dump())
    assert data == bson.encode(sp.model_dump())
    back = B.parameters_from_bson(data)
    assert isinstance(back.blob, bytes)  # the parameter store hands out a copy, like the reference
    assert back == SerializedParameters.model_validate(bson.decode(data))


def test_store_holds_bson_and_returns_views():
    from fedlesscan_amd.store import InMemoryClientResultStore, InMemoryParameterStore
    st_ = InMemoryClientResultStore()
    cr, layers = _result(1)
    st_.save("s", 2, "c", cr)
    assert st_._files[1] == bson.encode(cr.model_dump())  # what GridFS holds (client_daos.py:73)
    st_.save("s", 2, "d", bson.decode(bson.encode(cr.model_dump())))  # a dict is stored as given
    _, it = st_.load_results_for_round("s", 2)
    got = list(it)
    assert [g.cardinality for g in got] == [101, 101]
    assert all(isinstance(g.parameters.blob, memoryview) for g in got)
    ps = InMemoryParameterStore()
    ps.save("s", 3, cr.parameters)
    assert ps.load_latest("s").blob == cr.parameters.blob


def test_truncations_and_mutations_rejected_like_pymongo():
    cr, _ = _result(2, b64=False)
    seed = B.encode(cr.model_dump())
    for cut in range(len(seed)):
        with pytest.raises(B.InvalidBSON):
            B.decode(seed[:cut])
    rng = random.Random(5)
    agree = 0
    for _ in range(3000):
        c = bytearray(seed)
        for _ in range(rng.randint(1, 3)):
            c[rng.randrange(len(c))] = rng.randrange(256)
        c = bytes(c)
        try:
            ref = bson.decode(c)
        except Exception:
            ref = None
        try:
            got = B.decode(c)
        except B.InvalidBSON:
            got = None
        if ref is None:
            assert got is None  # pymongo rejects -> so do we
        elif got is not None:
            assert _same(got, ref)
            agree += 1
    assert agree > 100


@pytest.mark.parametrize("doc", [
    {"r": bson.Regex("a", "")}, {"c": bson.Code("f()")}, {"d": bson.Decimal128("1.5")},
])
def test_unused_types_raise(doc):
    with pytest.raises(B.InvalidBSON):
        B.decode(bson.encode(doc))


def test_encode_errors():
    with pytest.raises(B.InvalidDocument):
        B.encode({"a\x00": 1})
    with pytest.raises(B.InvalidDocument):
        B.encode({"a": np.float32(1)})
    with pytest.raises(B.InvalidDocument):
        B.encode({1: 1})
    with pytest.raises(OverflowError):
        B.encode({"a": 1 << 64})


def test_types_round_trip():
    d = {"i64": bson.Int64(5), "b2": bson.Binary(b"zz", 2), "b5": bson.Binary(b"q", 5),
         "oid": bson.ObjectId(b"abcdefghijkl"), "ts": bson.Timestamp(7, 9)}
    data = bson.encode(d)
    got = B.decode(data)
    assert got["i64"] == 5 and isinstance(got["i64"], B.Int64)
    assert got["b2"] == B.Binary(b"zz", 2) and got["b5"].subtype == 5
    assert bytes(got["oid"]) == b"abcdefghijkl" and got["ts"] == (7, 9)
    assert B.encode({k: got[k] for k in ("i64", "b5")}) == bson.encode({k: d[k] for k in ("i64", "b5")})
