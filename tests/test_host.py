"""CPU-side tests: the C-ABI library loads and exports its header, host-side
factor rounding, store/selection semantics, serialization, and the handler's
bookkeeping.  No GPU compute here (the GPU parity tests are in
test_gpu_parity.py)."""
import ctypes
import io

import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import _lib, engine
from fedlesscan_amd.aggregator.fed_avg_aggregator import chunked, resolve_cardinality
from fedlesscan_amd.common.models import (AggregationHyperParams, AggregationStrategy, AggregatorFunctionParams,
                                          BinaryStringFormat, ClientResult, NpzWeightsSerializerConfig,
                                          SerializedParameters, TestMetrics, WeightsSerializerConfig)
from fedlesscan_amd.common.serialization import (Base64StringConverter, NpzWeightsSerializer, SerializationError,
                                                 WeightsSerializerBuilder, deserialize_parameters)
from fedlesscan_amd.store import InMemoryClientResultStore, InMemoryParameterStore
from oracle import fedavg_oracle as O


# ---------------------------------------------------------------------------
# the C-ABI library
# ---------------------------------------------------------------------------
def test_library_exports_every_header_symbol():
    L = _lib.load()
    declared = _lib.header_functions()
    assert len(declared) >= 14
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    assert set(declared) == set(_lib._PROTOS), "ctypes prototypes out of sync with the header"
    assert L.fa_abi_version() == _lib.ABI_VERSION
    # the bench / tuning library exports its own header, and the product does not carry it
    B = _lib.load_bench()
    bench = _lib.header_functions(_lib.BENCH_HEADER)
    assert not [f for f in bench if not hasattr(B, f)]
    assert set(bench) == set(_lib._BENCH_PROTOS)
    assert not set(bench) & set(declared)
    assert not [f for f in bench if hasattr(L, f)], "tuning entry points leaked into the product library"


def test_product_library_exports_only_the_header():
    """`nm -D`: every exported fa_* symbol of libfedavg_hip.so is declared in
    include/fedavg_hip.h (no tuning scaffolding in the product ABI)."""
    import shutil
    import subprocess
    nm = shutil.which("nm") or shutil.which("llvm-nm")
    if nm is None:
        pytest.skip("no nm")
    out = subprocess.run([nm, "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("fa_")}
    assert exported == set(_lib.header_functions())


def test_library_variant_table():
    L = _lib.load_bench()
    n = L.fa_num_variants()
    assert n >= 1
    names = [L.fa_variant_name(i).decode() for i in range(n)]
    assert all(names) and len(set(names)) == n
    assert L.fa_variant_name(n) == b""


# The fp32 auto fold's kernel form by shape on a 256-CU MI355X:
# the BASELINE configs and the shapes whose sweeps set each boundary.
_PICKS = [
    ((1024, 10_000_000), "gs_bands_16k"),  # C3 (headline)
    ((100, 1_000_000), "tile_16k_ps"),     # C2: 245 tiles, 48+ clients at 0.7-1 tiles per CU
    ((512, 25_000_000), "gs_bands_16k"),   # C5
    ((256, 12_500_000), "gs_bands_16k"),   # a C4 bucket as fp32
    ((10, 582_026), "tile_4k"),            # C1 (config 1's MNIST CNN)
    ((32, 1_000_000), "tile_4k"),          # < 64 clients below one tile per CU
    ((200, 600_000), "tile_4k"),           # < 0.7 tiles per CU
    ((100, 582_026), "column"),            # 48-111 clients, < 0.6 tiles per CU
    ((64, 786_000), "tile_16k_ps"),        # 48+ clients at 0.7-1 tiles per CU (round 3)
    ((100, 786_000), "tile_16k_ps"),
    ((1024, 786_000), "tile_16k_ps"),
    ((40, 786_000), "tile_4k"),            # < 48 clients at 0.7-0.9
    ((64, 600_000), "column"),             # 48-79 clients below 0.7 tiles per CU
    ((1024, 1_000_000), "tile_16k_ps"),
    ((100, 1_500_000), "gs_bal_8k"),       # 1-2 tiles per CU
    ((1024, 582_026), "lds_w8_t32"),       # 256+ clients below 0.7
    ((10, 10_000_000), "tile_16k"),        # < 24 clients above one tile per CU
    ((1024, 16_384), "lds_w2_t16"),        # <= 16K params: six chunks in flight
    ((1024, 16_388), "lds_w2_t16_d4"),     # 16K-32K params: four
    ((1024, 67_267), "lds_w4_t24"),        # 32K-80K: CU-fill tile
    ((1024, 32_768), "lds_w2_t16_d4"),
    ((1024, 32_772), "lds_w4_t40"),
    ((1024, 65_536), "lds_w2_t16_d2"),
    ((256, 57_344), "lds_w2_t16_d2"),
    ((1024, 40_003), "lds_w4_t40"),
    ((1024, 131_072), "lds_w2_t32"),       # 80K-256K
]


@pytest.mark.parametrize("shape,pick", _PICKS)
def test_f32_auto_pick_table(shape, pick):
    B = _lib.load_bench()
    N, P = shape
    assert B.fa_f32_pick_name(N, P, 256).decode() == pick
    assert B.fa_f32_pick_name(0, P, 256) == b""


def test_library_argument_errors_need_no_gpu():
    L = _lib.load()
    # validation happens before any HIP call
    assert L.fa_fedavg_f32(None, 0, 10, 10, None, None, 1.0, None, None) == _lib.FA_ERR_NO_CLIENTS
    assert "N == 0" in _lib.last_error()
    assert L.fa_fedavg_f32(ctypes.c_void_p(16), 2, 10, 5, ctypes.c_void_p(16), None, 1.0,
                           ctypes.c_void_p(16), None) == _lib.FA_ERR_SHAPE
    assert L.fa_fedavg_f32(None, 2, 10, 10, None, None, 1.0, None, None) == _lib.FA_ERR_ARG
    assert L.fa_fedavg_f32(None, -1, 10, 10, None, None, 1.0, None, None) == _lib.FA_ERR_ARG
    with pytest.raises(Exception) as ei:
        _lib.check(_lib.FA_ERR_NO_CLIENTS, "x")
    assert type(ei.value).__name__ == "InsufficientClientResults"


def test_exchange_entry_argument_errors_need_no_gpu():
    """The multi-GPU entries validate before any HIP call: bad peer-group
    shapes, null handles, malformed step-form keys (ABI 5: no peer fence; the
    rounds entries with host factors)."""
    L = _lib.load()
    h = ctypes.c_void_p()
    for world, rank, nbytes in ((0, 0, 64), (17, 0, 64), (2, 2, 64), (2, -1, 64), (2, 0, 8), (2, 0, 100)):
        assert L.fa_peers_create(ctypes.byref(h), 0, world, rank, nbytes) == _lib.FA_ERR_ARG, (world, rank, nbytes)
        assert h.value is None
    assert L.fa_peers_create(None, 0, 2, 0, 64) == _lib.FA_ERR_ARG
    assert L.fa_peers_handle_bytes() == 2 * 64  # two hipIpcMemHandle_t: the send buffers, the signal words
    assert "fa_peers_fence" not in _lib.header_functions()  # ABI 5: the double-buffered exchange needs none
    assert L.fa_fedavg_f32_rounds_hostf(None, None, 1, 4, None, None, 1.0, None, 1, None, None, None) == \
        _lib.FA_ERR_ARG
    assert L.fa_fedavg_bf16_rounds_hostf(None, None, 1, 8, None, None, 1.0, None, None, 1, None, None, None) == \
        _lib.FA_ERR_ARG
    assert L.fa_peers_exchange(None, 1, None, None, None, None) == _lib.FA_ERR_ARG
    assert L.fa_peers_send(None) is None and L.fa_peers_rounds(None) is None
    assert L.fa_peers_destroy(None) == _lib.FA_OK
    assert L.fa_rounds_check(None) < 0
    assert L.fa_step_lookup(b"gfx950:256 f16 8 256 100 64") == -2
    assert L.fa_step_lookup(b"gfx950:256 bf16 8 255 100 64") == -2
    assert L.fa_step_lookup(None) == -2
    assert L.fa_step_record(b"not a key", 1) == _lib.FA_ERR_ARG


def test_product_package_does_not_import_oracle():
    import pathlib
    pkg = pathlib.Path(_lib.PKG)
    for f in pkg.rglob("*.py"):
        text = f.read_text()
        assert "import oracle" not in text and "from oracle" not in text, f


# ---------------------------------------------------------------------------
# numpy-exact host factors
# ---------------------------------------------------------------------------
def test_result_dtype_matches_numpy():
    cases = [(np.float32, [1, 2, 3], None), (np.float32, [1.5, 2], None), (np.float32, [1, 2], [0.5, 1.0]),
             (np.float64, [3, 4], None), (np.int64, [1, 2], None), (np.int32, [1, 2], None),
             (np.int64, [1.5, 2], None), (np.float32, [np.int64(3), 2], None)]
    for dt, w, s in cases:
        xs = [np.ones(3, dtype=dt) for _ in w]
        ref = (O.fedavg_literal([[x] for x in xs], w) if s is None else
               O.stall_aware_literal([{"round_id": 0}] * len(w), 0, [[x] for x in xs], w))
        assert engine.result_dtype(np.dtype(dt), w, s) == ref[0].dtype, (dt, w, s)


def test_factors_round_like_numpy():
    w = [3, 16777217, 2.5, 0.1]
    f = engine.Factors(w, [1 / 3, 2 / 3, 0.7, 1.0], np.dtype(np.float32))
    for x, aw in zip(w, f.a):
        assert aw == (np.ones(1, np.float32) * x)[0]
    assert f.div == (np.ones(1, np.float32) / np.float32(1) * 0 + np.float32(sum(w)))[0]
    assert f.s[0] == (np.ones(1, np.float32) * (1 / 3))[0]


def test_weak_f32_helper_matches_numpy():
    """The C rounding helper (hostfast.c) gives numpy's float32 of every weak
    Python scalar bit for bit, and declines (None) whatever numpy would treat
    differently; Factors.weak_f32 then equals the general Factors."""
    assert engine._hostfast is not None, "native build did not produce _hostfast"

    class F(float):
        pass

    rng = np.random.default_rng(3)
    floats = [float(x) for x in rng.standard_normal(300) * 10.0 ** rng.integers(-45, 40, 300)]
    floats += [0.0, -0.0, float("inf"), -float("inf"), 1e39, -1e39, 5e-324, 1.4e-45, 7e-46, 3.4028235e38,
               3.4028236e38, 0.1, 1 / 3, 16777217.0]
    ints = [int(x) for x in rng.integers(-2 ** 52, 2 ** 52, 200)] + [0, 1, -1, 16777217, 2 ** 53 - 1, -(2 ** 53 - 1)]
    vals = floats + ints + [True, False]
    got = engine.weak_f32(vals)
    exp = np.array([np.float32(v) for v in vals], dtype=np.float32)
    assert got.view(np.uint32).tolist() == exp.view(np.uint32).tolist()
    nan = engine.weak_f32([float("nan")])
    assert np.isnan(nan[0])
    assert engine.weak_f32(tuple(ints)).tolist() == [np.float32(v) for v in ints]
    assert engine.weak_f32([]).size == 0
    for bad in ([1, 2 ** 53], [1, -(2 ** 53)], [2 ** 70], [np.float64(1.0)], [np.int64(3)], [1, F(2.0)],
                [1, "2"], [1, None], [np.float32(1)]):
        assert engine.weak_f32(bad) is None, bad
    w, sc = [3, 16777217, 2.5, 0.1, True], [1 / 3, 2 / 3, 0.7, 1.0, 0.5]
    fw, fg = engine.Factors.weak_f32(w, sc), engine.Factors(w, sc, np.dtype(np.float32))
    assert fw.a.tobytes() == fg.a.tobytes() and fw.s.tobytes() == fg.s.tobytes()
    assert np.float32(fw.div).tobytes() == np.float32(fg.div).tobytes() and fw.total == fg.total
    assert engine.Factors.weak_f32(w, None, total=np.int64(7)) is None
    assert engine.Factors.weak_f32([np.float64(1.0)], None) is None


def test_cardinality_resolution_quirks():
    from fedlesscan_amd import UnknownCardinalityError
    assert resolve_cardinality(5, None) == 5
    assert resolve_cardinality(-1, 2.0) == 2.0
    with pytest.raises(UnknownCardinalityError):
        resolve_cardinality(-2, None)
    with pytest.raises(UnknownCardinalityError):  # `if not default_cardinality`: 0.0 counts as absent
        resolve_cardinality(-1, 0.0)


def test_chunking_matches_reference_semantics():
    assert [len(c) for c in chunked(range(7), 3)] == [3, 3, 1]
    assert [len(c) for c in chunked(range(6), 3)] == [3, 3]
    assert list(chunked([], 3)) == []


# ---------------------------------------------------------------------------
# serialization (mirrors reference test/test_serialize.py:198-299)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("compressed", [True, False])
def test_npz_roundtrip_and_types(compressed):
    s = NpzWeightsSerializer(compressed=compressed)
    w = [np.random.randn(10, 15).astype(np.float32), np.random.randint(0, 32, (8, 5)),
         np.random.randint(0, 1, (5, 6)).astype(np.int8)]
    r = s.deserialize(s.serialize(w))
    assert all(np.array_equal(a, b) and a.dtype == b.dtype for a, b in zip(w, r))
    assert s.deserialize(s.serialize([])) == []


def test_npz_errors_wrap():
    with pytest.raises(SerializationError):
        NpzWeightsSerializer().deserialize(b"")
    with pytest.raises(SerializationError):
        NpzWeightsSerializer().deserialize(b"not a zip at all")


def test_deserialize_parameters_formats():
    w = [np.random.rand(10, 10, 15), np.random.rand(99, 4, 3)]
    blob = NpzWeightsSerializer(compressed=True).serialize(w)
    sp = SerializedParameters(blob=Base64StringConverter.to_str(blob),
                              serializer=WeightsSerializerConfig(type="npz",
                                                                 params=NpzWeightsSerializerConfig(compressed=True)),
                              string_format=BinaryStringFormat.BASE64)
    assert all(np.array_equal(a, b) for a, b in zip(deserialize_parameters(sp), w))
    sp = SerializedParameters(blob=NpzWeightsSerializer().serialize(w),
                              serializer=WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig()))
    assert all(np.array_equal(a, b) for a, b in zip(deserialize_parameters(sp), w))
    with pytest.raises(NotImplementedError):
        WeightsSerializerBuilder.from_config(WeightsSerializerConfig.model_construct(type="h5", params=None))


# ---------------------------------------------------------------------------
# store: selection order, tolerance window, counts (client_daos.py:150-235)
# ---------------------------------------------------------------------------
def _cr(v, card=10):
    blob = NpzWeightsSerializer().serialize([np.full(4, v, np.float32)])
    return ClientResult(parameters=SerializedParameters(
        blob=blob, serializer=WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())),
        cardinality=card)


def test_store_selection_semantics():
    st = InMemoryClientResultStore()
    for r in (7, 8, 9, 10):
        for c in ("a", "b"):
            st.save("s", r, c, _cr(r))
    st.save("other", 10, "a", _cr(0))
    st.save("s", 8, "a", _cr(88))  # upsert keeps its position
    d, it = st.load_results_for_round("s", 10)
    assert [x["client_id"] for x in d] == ["a", "b"]
    d, it = st.load_results_for_session("s", 10, tolerance=2)
    assert [(x["round_id"], x["client_id"]) for x in d] == [(8, "a"), (8, "b"), (9, "a"), (9, "b"),
                                                             (10, "a"), (10, "b")]
    first = next(it)
    assert deserialize_parameters(first.parameters)[0][0] == 88
    assert st.count_results_for_round("s", 10) == 2
    assert st.count_results_for_session("s") == 8  # whole session, not the window
    st.delete_results_for_round("s", 10)
    assert st.count_results_for_session("s") == 6
    st.delete_results_for_session("s")
    assert st.count_results_for_session("s") == 0 and st.count_results_for_session("other") == 1


def test_store_returns_fresh_objects():
    st = InMemoryClientResultStore()
    st.save("s", 1, "a", _cr(1))
    _, it = st.load_results_for_round("s", 1)
    r = next(it)
    r.parameters = None
    _, it = st.load_results_for_round("s", 1)
    assert next(it).parameters is not None


# ---------------------------------------------------------------------------
# handler bookkeeping (aggregation.py:45-167) with the fold supplied by the
# oracle (these tests check selection / counts / persistence, not numerics)
# ---------------------------------------------------------------------------
@pytest.fixture
def oracle_fold(monkeypatch):
    def fake(parameters, weights, scores=None, device=None, devices=None):
        n = min(len(parameters), len(weights), len(scores) if scores is not None else len(weights))
        if scores is None:
            return O.fedavg_literal(parameters[:n], list(weights))
        return _stall(parameters[:n], list(weights), list(scores))
    def fake_decoded(items, scores=None, device=None, devices=None, expected_rows=0):
        rows, ws = [], []
        for layers, w in items:
            rows.append(layers)
            ws.append(w)
        return fake(rows, ws, scores) if rows else []
    monkeypatch.setattr(engine, "aggregate_layers", fake)
    monkeypatch.setattr(engine, "aggregate_decoded", fake_decoded)


def _stall(params, weights, scores):
    """stall-aware fold with explicit scores (the oracle derives them from round ids)."""
    from functools import reduce
    total = sum(weights)
    prods = [[np.multiply(np.multiply(l, n), s) for l in p] for p, n, s in zip(params, weights, scores)]
    return [reduce(np.add, ls) / total for ls in zip(*prods)]


def test_handler_per_round(oracle_fold):
    from fedlesscan_amd.handler import MockAggregator
    st, ps = InMemoryClientResultStore(), InMemoryParameterStore()
    for i in range(10):
        st.save("sess", 3, f"c{i}", _cr(float(i), card=6000))
    st.save("sess", 2, "old", _cr(100.0))
    res = MockAggregator(AggregatorFunctionParams(session_id="sess", round_id=3), st, ps).run_aggregator()
    assert res.new_round_id == 4 and res.num_clients == 10
    out = NpzWeightsSerializer().deserialize(ps.load("sess", 4).blob)
    assert out[0][0] == np.float32(4.5)
    assert st.count_results_for_round("sess", 3) == 0 and st.count_results_for_session("sess") == 1


def test_handler_per_session_tolerance(oracle_fold):
    from fedlesscan_amd.handler import default_aggregation_handler
    st, ps = InMemoryClientResultStore(), InMemoryParameterStore()
    st.save("s", 7, "stale", _cr(1000.0))  # outside R - tol
    st.save("s", 8, "a", _cr(1.0))
    st.save("s", 10, "b", _cr(2.0))
    hp = AggregationHyperParams(tolerance=2)
    cfg = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())
    res = default_aggregation_handler("s", 10, st, ps, cfg, None, True, AggregationStrategy.PER_SESSION, hp)
    assert res.new_round_id == 11
    assert res.num_clients == 3  # count_results_for_session counts every session result
    out = NpzWeightsSerializer().deserialize(ps.load_latest("s").blob)[0]
    exp = (np.float32(1.0) * 10 * (9 / 11) + np.float32(2.0) * 10 * (11 / 11)) / 20
    assert out[0] == pytest.approx(exp, rel=1e-6)
    assert st.count_results_for_session("s") == 0


def test_handler_no_results_saves_empty_model(oracle_fold):
    # the reference never raises InsufficientClientResults at selection (it tests a
    # generator's truthiness, fed_avg_aggregator.py:51-54): an empty round saves []
    # at R+1 and reports num_clients=0 (pinned in test_handler_golden.py)
    from fedlesscan_amd.handler import default_aggregation_handler
    cfg = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())
    ps = InMemoryParameterStore()
    res = default_aggregation_handler("s", 1, InMemoryClientResultStore(), ps, cfg)
    assert res.new_round_id == 2 and res.num_clients == 0 and res.test_results is None
    assert NpzWeightsSerializer().deserialize(ps.load("s", 2).blob) == []


def test_handler_online_uses_stream_variant(oracle_fold):
    from fedlesscan_amd.handler import default_aggregation_handler
    st, ps = InMemoryClientResultStore(), InMemoryParameterStore()
    for i in range(30):
        st.save("s", 1, f"c{i}", _cr(float(i), card=i + 1))
    cfg = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())
    res = default_aggregation_handler("s", 1, st, ps, cfg, None, False, AggregationStrategy.PER_ROUND,
                                      AggregationHyperParams(aggregate_online=True))
    assert res.num_clients == 30 and st.count_results_for_round("s", 1) == 30
    out = NpzWeightsSerializer().deserialize(ps.load("s", 2).blob)[0]
    params = [[np.full(4, float(i), np.float32)] for i in range(30)]
    results = [{"blob": NpzWeightsSerializer().serialize(p), "cardinality": i + 1} for i, p in enumerate(params)]
    exp = O.aggregate_stream_fedavg(results, 25)[0][0]
    assert np.array_equal(out, exp)


def test_test_metrics_are_collected(oracle_fold):
    from fedlesscan_amd import FedAvgAggregator
    crs = [_cr(1.0), _cr(2.0)]
    crs[0].test_metrics = TestMetrics(cardinality=5, metrics={"loss": 1.0})
    _, metrics = FedAvgAggregator().aggregate(crs, None)
    assert len(metrics) == 1 and metrics[0].cardinality == 5
    assert crs[0].parameters is None  # blob released after decode, as the reference does


# ---------------------------------------------------------------------------
# zero-copy NPZ reader (fedlesscan_amd/npz.py) == np.load
# ---------------------------------------------------------------------------
def _savez(layers, compressed=False):
    f = io.BytesIO()
    (np.savez_compressed if compressed else np.savez)(f, *layers)
    return f.getvalue()


def test_npz_views_match_np_load():
    from fedlesscan_amd.npz import npz_views, read_layers
    layers = [np.arange(12, dtype=np.float32).reshape(3, 4), np.float32(3.5) * np.ones(()),
              np.zeros((0, 5), np.float32), np.arange(7, dtype=np.int64), np.ones((2, 2, 2), np.float64),
              np.arange(1000, dtype=np.float32)[::1]]
    blob = _savez(layers)
    v = npz_views(blob)
    assert v is not None and len(v) == len(layers)
    for a, b in zip(v, layers):
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)
    # views alias the blob (no copy)
    assert all(not x.flags.owndata for x in v)
    # compressed and Fortran-ordered members fall back to np.load
    assert npz_views(_savez(layers, compressed=True)) is None
    assert npz_views(_savez([np.asfortranarray(np.ones((3, 4), np.float32))])) is None
    for blob2 in (_savez(layers, compressed=True), _savez([np.asfortranarray(np.ones((3, 4), np.float32))])):
        ref = [np.load(io.BytesIO(blob2))[k] for k in np.load(io.BytesIO(blob2)).files]
        got = read_layers(blob2)
        assert all(np.array_equal(a, b) for a, b in zip(got, ref))
    assert npz_views(b"junk") is None
    assert npz_views(_savez([])) == []


# ---------------------------------------------------------------------------
# BASELINE config 1: mnist-demo (aggregator tolerance 2), 10 clients, mock
# aggregator.  Plumbing checked against the reference-generated golden with the
# oracle supplying the fold (the GPU version of this test is in test_gpu_parity).
# ---------------------------------------------------------------------------
def config1_round(strategy_name, pinned=False):
    """Store the 10 mnist-demo client results, run one MockAggregator round,
    return (result, output shapes, sha256 of the flat output, golden entry).
    pinned=True keeps the stored documents in page-locked memory (GPU only)."""
    import hashlib
    from fedlesscan_amd.config import aggregator_settings
    from fedlesscan_amd.handler import MockAggregator
    m = G.manifest()["mnist_c1"]
    strategy, hp = aggregator_settings({"aggregator": {"hyperparams": {"tolerance": 2}}}, strategy_name)
    st, ps = InMemoryClientResultStore(pinned=pinned), InMemoryParameterStore()
    params = G.parameters("mnist_c1")
    rounds = m["round_ids"] if strategy == AggregationStrategy.PER_SESSION else [m["current_round"]] * 10
    for i, (p, r) in enumerate(zip(params, rounds)):
        blob = NpzWeightsSerializer().serialize(p)
        st.save("mnist", r, f"client-{i}", ClientResult(parameters=SerializedParameters(
            blob=blob, serializer=WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())),
            cardinality=m["weights"][i]))
    res = MockAggregator(AggregatorFunctionParams(session_id="mnist", round_id=m["current_round"],
                                                  aggregation_strategy=strategy, aggregation_hyper_params=hp),
                         st, ps).run_aggregator()
    out = NpzWeightsSerializer().deserialize(ps.load("mnist", m["current_round"] + 1).blob)
    flat = np.concatenate([o.ravel() for o in out])
    key = "stall" if strategy == AggregationStrategy.PER_SESSION else "fedavg"
    return res, [o.shape for o in out], hashlib.sha256(flat.tobytes()).hexdigest(), m["outputs"][key]


@pytest.mark.parametrize("strategy_name", ["fedlesscan", "fedavg"])
def test_config1_mock_aggregator_plumbing(oracle_fold, strategy_name):
    res, shapes, sha, exp = config1_round(strategy_name)
    assert res.new_round_id == 11 and res.num_clients == 10
    assert [list(s) for s in shapes] == exp["shapes"]
    assert sha == exp["flat_sha256"]


def test_strategy_name_mapping():
    from fedlesscan_amd.config import strategy_for
    assert strategy_for("fedlesscan") == AggregationStrategy.PER_SESSION
    assert strategy_for("fedavg") == AggregationStrategy.PER_ROUND
    assert strategy_for("fedprox") == AggregationStrategy.PER_ROUND
    assert strategy_for("unknown") == AggregationStrategy.PER_SESSION


def test_native_npz_index_matches_python_and_np_load():
    from fedlesscan_amd.npz import native_views, npz_views
    rng = np.random.default_rng(5)
    cases = [
        [np.arange(12, dtype=np.float32).reshape(3, 4), np.zeros((0, 5), np.float32)],
        [np.float32(3.5) * np.ones(()), np.arange(7, dtype=np.int64), np.ones((2, 2, 2), np.float64)],
        [rng.standard_normal((5, 5, 1, 32)).astype(np.float32), rng.standard_normal(32).astype(np.float32),
         rng.integers(0, 9, (4, 3)).astype(np.int32), np.array([True, False]), np.arange(5, dtype=np.int8),
         np.arange(6, dtype=np.uint8), np.ones(3, np.float16)],
        [],
    ]
    for layers in cases:
        blob = _savez(layers)
        nv, pv = native_views(blob), npz_views(blob)
        assert nv is not None and pv is not None and len(nv) == len(pv) == len(layers)
        for a, b, c in zip(nv, pv, layers):
            assert a.dtype == b.dtype == np.asarray(c).dtype and a.shape == b.shape == np.asarray(c).shape
            assert np.array_equal(a, c) and not a.flags.owndata
    assert native_views(_savez([np.ones(3, np.float32)], compressed=True)) is None
    assert native_views(_savez([np.asfortranarray(np.ones((3, 4), np.float32))])) is None
    assert native_views(_savez([np.ones(3, dtype=">f4")])) is None
    assert native_views(b"not a zip") is None


def test_native_npz_index_survives_corruption():
    from fedlesscan_amd.npz import native_views
    blob = bytearray(_savez([np.arange(100, dtype=np.float32), np.ones((3, 3), np.float64)]))
    rng = np.random.default_rng(9)
    for cut in range(0, len(blob), 37):  # truncations
        native_views(bytes(blob[:cut]))
    for _ in range(300):  # single-byte mutations: never crash, never read out of bounds
        b = bytearray(blob)
        b[rng.integers(0, len(b))] = rng.integers(0, 256)
        v = native_views(bytes(b))
        if v is not None:
            assert sum(x.nbytes for x in v) <= len(b)


def test_fa_crc32_matches_zlib():
    """The NPZ writer's checksum: zlib.crc32 for any length, alignment,
    starting value and thread count (threaded ranges joined by the combine)."""
    import zlib
    L = _lib.load()
    out = ctypes.c_uint32()
    buf = np.random.default_rng(11).integers(0, 256, size=9_000_000, dtype=np.uint8)
    for n in (0, 1, 7, 15, 16, 17, 63, 4099, (1 << 21) - 1, (1 << 21) + 5, 4_500_001, 8_999_990):
        for off in (0, 1, 5):
            for crc_in in (0, 0x9E3779B9):
                for T in (1, 3, 16):
                    v = buf[off:off + n]
                    assert L.fa_crc32(v.ctypes.data if n else None, n, crc_in, T, ctypes.byref(out)) == 0
                    assert out.value == zlib.crc32(v.tobytes(), crc_in), (n, off, crc_in, T)
    assert L.fa_crc32(None, 5, 0, 1, ctypes.byref(out)) == _lib.FA_ERR_ARG
    assert "fa_crc32" in _lib.last_error()  # the host entries set the error text too
    assert L.fa_pack(None, None, None, None, 3, 1) == _lib.FA_ERR_ARG
    assert "fa_pack" in _lib.last_error()


def test_npz_writer_is_byte_identical_to_savez():
    """write_npz (and so NpzWeightsSerializer.serialize, uncompressed) returns
    exactly np.savez's bytes; layouts numpy writes differently fall back."""
    from fedlesscan_amd.npz import write_npz
    rng = np.random.default_rng(12)

    def savez(arrs):
        f = io.BytesIO()
        np.savez(f, *arrs)
        return f.getvalue()

    cases = [
        [],
        [np.arange(5, dtype=np.float32)],
        [rng.random((3, 4)).astype(np.float32), np.ones(()), np.zeros((0, 3), np.float32)],
        [rng.integers(0, 9, (2, 3, 4)), np.array([True, False]), rng.random(7).astype(np.float16),
         np.array(5, dtype=np.int32), rng.random(3).astype(">f4")],
        [np.zeros((2, 2), dtype=[("a", "<f4"), ("b", "<i8")])],
        [rng.random(n).astype(np.float32) for n in (1, 31, 32, 33, 4096, 1_000_003)],
        [np.asfortranarray(rng.random((2, 3)))[:, :1].copy()],
    ]
    for arrs in cases:
        assert write_npz(arrs) == savez(arrs), [a.shape for a in arrs]
        assert NpzWeightsSerializer().serialize(arrs) == savez(arrs)
    for odd in ([rng.random((3, 5)).T], [np.array([1, "a"], dtype=object)], [rng.random(10)[::2]]):
        assert write_npz(odd) is None
        assert NpzWeightsSerializer().serialize(odd) == savez(odd)
    # and it reads back through both readers
    arrs = cases[3]
    blob = write_npz(arrs)
    assert all(np.array_equal(a, b) for a, b in zip(NpzWeightsSerializer().deserialize(blob), arrs))


def test_fa_pack_scatters_ranges():
    L = _lib.load()
    rng = np.random.default_rng(3)
    srcs = [rng.integers(0, 255, rng.integers(0, 5_000_000), dtype=np.uint8) for _ in range(9)]
    offs, pos = [], 0
    for s in srcs:
        pos += int(rng.integers(0, 100))
        offs.append(pos)
        pos += s.size
    dst = np.zeros(pos + 10, np.uint8)
    ptrs = np.array([s.ctypes.data for s in srcs], np.uint64)
    sizes = np.array([s.size for s in srcs], np.int64)
    o = np.array(offs, np.int64)
    for threads in (1, 3, 0):
        dst[:] = 0
        assert L.fa_pack(dst.ctypes.data, o.ctypes.data, ptrs.ctypes.data, sizes.ctypes.data, len(srcs), threads) == 0
        for s, off in zip(srcs, offs):
            assert np.array_equal(dst[off:off + s.size], s)
    assert L.fa_pack(None, None, None, None, -1, 1) == _lib.FA_ERR_ARG


def test_aggregate_metrics_matches_oracle():
    from fedlesscan_amd.metrics import aggregate_metrics
    raw = [{"cardinality": 10, "metrics": {"loss": 1.0, "accuracy": 0.5}},
           {"cardinality": 30, "metrics": {"loss": 3.0, "accuracy": 0.9}},
           {"cardinality": 7, "metrics": {"loss": 0.25, "accuracy": 0.1}}]
    got = aggregate_metrics([TestMetrics(**r) for r in raw], ["loss", "accuracy"])
    exp = O.weighted_metrics(raw, ["loss", "accuracy"])
    assert got == exp


def test_handler_wraps_serialization_errors(oracle_fold):
    from fedlesscan_amd import AggregationError
    from fedlesscan_amd.handler import default_aggregation_handler
    st, ps = InMemoryClientResultStore(), InMemoryParameterStore()
    bad = ClientResult(parameters=SerializedParameters(
        blob=b"definitely not an npz", serializer=WeightsSerializerConfig(type="npz",
                                                                          params=NpzWeightsSerializerConfig())),
        cardinality=3)
    st.save("s", 1, "c0", bad)
    cfg = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())
    with pytest.raises(AggregationError):  # aggregation.py:164-165
        default_aggregation_handler("s", 1, st, ps, cfg)
    assert st.count_results_for_round("s", 1) == 1  # nothing deleted on failure


def test_aggregator_settings_from_yaml(tmp_path):
    from fedlesscan_amd.config import aggregator_settings
    p = tmp_path / "exp.yaml"
    p.write_text("aggregator:\n  hyperparams:\n    tolerance: 2\n    aggregate_online: true\n"
                 "  function:\n    params: {type: openfaas, url: http://x}\n    type: openfaas\n"
                 "clients:\n  hyperparams: {epochs: 5}\n")
    strategy, hp = aggregator_settings(str(p), "fedlesscan")
    assert strategy == AggregationStrategy.PER_SESSION
    assert hp.tolerance == 2 and hp.aggregate_online is True and hp.test_batch_size == 10
    strategy, hp = aggregator_settings({}, "fedavg")
    assert strategy == AggregationStrategy.PER_ROUND and hp.tolerance == 0


# ---------------------------------------------------------------------------
# FaaS entry points (functions/aggregator_functions/*, providers.py)
# ---------------------------------------------------------------------------
def _stores_with_round(n=4, round_id=3, session="s"):
    st, ps = InMemoryClientResultStore(), InMemoryParameterStore()
    rng = np.random.default_rng(5)
    for i in range(n):
        p = [rng.standard_normal((2, 3)).astype(np.float32), rng.standard_normal(4).astype(np.float32)]
        st.save(session, round_id, f"c{i}", ClientResult(parameters=SerializedParameters(
            blob=NpzWeightsSerializer().serialize(p),
            serializer=WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())),
            cardinality=i + 1))
    return st, ps


REF_REQUEST = {  # what the reference controller sends (aggregation_models.py:25-34)
    "session_id": "s", "round_id": 3,
    "database": {"host": "mongo", "port": 27017, "username": "u", "password": "p"},
    "serializer": {"type": "npz", "params": {"type": "npz", "compressed": False}},
    "test_data": None,
    "aggregation_hyper_params": {"tolerance": 0, "aggregate_online": False, "test_batch_size": 10},
    "aggregation_strategy": "per_round",
}


def test_openfaas_entry_point(oracle_fold):
    import json
    from fedlesscan_amd.functions import Event, make_openfaas_handler
    st, ps = _stores_with_round()
    handle = make_openfaas_handler(st, ps)
    resp = handle(Event(json.dumps(REF_REQUEST)), None)
    assert resp["statusCode"] == 200 and resp["headers"]["Content-Type"] == "application/json"
    body = json.loads(resp["body"])
    assert body == {"new_round_id": 4, "num_clients": 4, "test_results": None, "global_test_results": None}
    assert ps.load("s", 4) is not None
    # the round's results were deleted (delete_results_after_finish default): a second
    # call finds none and, as in the reference, saves an empty model with num_clients 0
    resp = handle(Event(json.dumps(REF_REQUEST)), None)
    assert resp["statusCode"] == 200
    assert json.loads(resp["body"]) == {"new_round_id": 4, "num_clients": 0, "test_results": None,
                                        "global_test_results": None}
    # an error -> 400 {errorMessage, errorType, details} (providers.py:25-40)
    resp = handle(Event(json.dumps(dict(REF_REQUEST, aggregation_strategy="bogus"))), None)
    err = json.loads(resp["body"])
    assert resp["statusCode"] == 400 and set(err) == {"errorMessage", "errorType", "details"}
    # malformed request -> pydantic ValidationError -> 400
    bad = dict(REF_REQUEST)
    del bad["round_id"]
    resp = handle(Event(json.dumps(bad)), None)
    assert resp["statusCode"] == 400 and json.loads(resp["body"])["errorType"] == "ValidationError"
    # global evaluation is out of scope -> AggregationError -> 400
    st, ps = _stores_with_round()
    req = dict(REF_REQUEST, test_data={"type": "mnist", "params": {}})
    resp = make_openfaas_handler(st, ps)(Event(json.dumps(req)))
    assert resp["statusCode"] == 400 and json.loads(resp["body"])["errorType"] == "AggregationError"


def test_openwhisk_entry_point(oracle_fold):
    import base64
    import json
    from fedlesscan_amd.functions import make_openwhisk_main
    st, ps = _stores_with_round()
    main = make_openwhisk_main(st, ps)
    resp = main(dict(REF_REQUEST))  # plain action: the params are the body
    assert resp["statusCode"] == 200 and json.loads(resp["body"])["num_clients"] == 4
    # web action: __ow_ keys, body base64-encoded JSON
    st, ps = _stores_with_round()
    main = make_openwhisk_main(st, ps)
    enc = base64.b64encode(json.dumps(REF_REQUEST).encode()).decode()
    resp = main({"__ow_body": enc, "__ow_method": "post", "__ow_headers": {}})
    assert resp["statusCode"] == 200 and json.loads(resp["body"])["new_round_id"] == 4
    # a body that is neither JSON nor base64 -> binascii.Error -> 400
    resp = main({"__ow_body": "abc", "__ow_method": "post"})
    assert resp["statusCode"] == 400 and json.loads(resp["body"])["errorType"] == "Error"


def test_serialize_without_the_native_library(monkeypatch):
    """A process that only saves a model needs no HIP library: write_npz
    declines and NpzWeightsSerializer.serialize falls back to np.savez (the
    same bytes)."""
    import io
    from fedlesscan_amd import npz
    from fedlesscan_amd.aggregator.exceptions import AggregationError
    from fedlesscan_amd.common.serialization import NpzWeightsSerializer

    def missing(*a, **k):
        raise AggregationError("HIP extension not built")

    monkeypatch.setattr(_lib, "load", missing)
    arrs = [np.arange(12, dtype=np.float32).reshape(3, 4), np.ones(5, np.float64)]
    assert npz.write_npz(arrs) is None
    f = io.BytesIO()
    np.savez(f, *arrs)
    assert NpzWeightsSerializer().serialize(arrs) == f.getvalue()
