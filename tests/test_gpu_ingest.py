"""GPU: host-side ingest routes into the fold (fedlesscan_amd/ingest.py).

Rows whose layers sit in page-locked memory are DMA'd straight from the stored
document (fa_copy_h2d); other rows are packed (fa_pack) and copied in runs.
Whatever the route and the mix, the fold must be bit-identical to the batch
fold and to the reference-generated goldens."""
import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth
from oracle import oracle_lib as OL  # checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def test_host_is_pinned(dev):
    from fedlesscan_amd.pinned import is_pinned, pinned_bytes
    t = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True)
    assert is_pinned(t.data_ptr(), t.numel())
    assert is_pinned(t.data_ptr() + 4096, 1000)
    a = np.zeros(1 << 20, np.uint8)  # pageable
    assert not is_pinned(a.ctypes.data, a.nbytes)
    v = pinned_bytes(12345)
    base = np.frombuffer(v, np.uint8).ctypes.data
    assert is_pinned(base, 12345) and not is_pinned(base, 1 << 30)
    v[:5] = b"hello"
    assert bytes(v[:5]) == b"hello"
    del v  # released with its last view


@pytest.mark.parametrize("chunk_rows", [1, 3, 16])
@pytest.mark.parametrize("pattern", ["all_pinned", "mixed", "none_pinned"])
@pytest.mark.parametrize("scored", [False, True])
def test_direct_and_packed_rows_mix(dev, chunk_rows, pattern, scored):
    from fedlesscan_amd.ingest import StreamingFold
    from fedlesscan_amd.pinned import pinned_bytes
    N, P = 23, 5003
    X = synth.clients_f32(97, N, 0, P)
    w = synth.cardinalities(97, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(97, N, 10, 2)] if scored else None
    rows = []
    for i in range(N):
        pin = pattern == "all_pinned" or (pattern == "mixed" and i % 3 != 1)
        if pin:
            buf = np.frombuffer(pinned_bytes(P * 4), np.float32)
            buf[:] = X[i]
            rows.append(buf)
        else:
            rows.append(X[i].copy())
    before = dict(StreamingFold.stats)
    sf = StreamingFold(P, chunk_rows=chunk_rows, device=dev, direct=True)
    sf.acc.fill_(float("nan"))
    for i in range(N):
        r = rows[i]
        sf.add([r[:1000].reshape(10, 100), r[1000:3000], r[3000:]], w[i], None if sc is None else sc[i])
    got = sf.finish().cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert G.same_bits(got, exp)
    n_direct = {"all_pinned": N, "mixed": sum(1 for i in range(N) if i % 3 != 1), "none_pinned": 0}[pattern]
    assert sf.direct_rows == n_direct
    assert StreamingFold.stats["direct_rows"] - before["direct_rows"] == n_direct


def test_direct_off_packs_everything(dev):
    from fedlesscan_amd.ingest import StreamingFold
    from fedlesscan_amd.pinned import pinned_bytes
    N, P = 5, 777
    X = synth.clients_f32(5, N, 0, P)
    w = synth.cardinalities(5, N)
    sf = StreamingFold(P, chunk_rows=2, device=dev, direct=False)
    for i in range(N):
        buf = np.frombuffer(pinned_bytes(P * 4), np.float32)
        buf[:] = X[i]
        sf.add(buf, w[i])
    got = sf.finish().cpu().numpy()
    assert sf.direct_rows == 0
    assert G.same_bits(got, OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w))))


@pytest.mark.parametrize("strategy_name", ["fedlesscan", "fedavg"])
def test_config1_pinned_store_direct_route(dev, strategy_name, monkeypatch):
    """BASELINE config 1 through a pinned result store with the direct DMA
    route on: every client row takes it, and the round is bit-exact against the
    reference's golden output."""
    from fedlesscan_amd import engine
    from fedlesscan_amd.ingest import StreamingFold
    monkeypatch.setattr(engine, "DIRECT_DMA", True)
    from test_host import config1_round
    before = StreamingFold.stats["direct_rows"]
    res, shapes, sha, exp = config1_round(strategy_name, pinned=True)
    assert res.new_round_id == 11 and res.num_clients == 10
    assert [list(s) for s in shapes] == exp["shapes"]
    assert sha == exp["flat_sha256"]
    assert StreamingFold.stats["direct_rows"] - before == 10


def test_pinned_bson_documents_round_trip(dev):
    from fedlesscan_amd import bsondoc as B
    from fedlesscan_amd.pinned import is_pinned, pinned_bytes
    d = {"parameters": {"blob": bytes(range(256)) * 100, "string_format": "none"}, "cardinality": 7}
    v = B.encode_into(d, pinned_bytes)
    assert bytes(v) == B.encode(d)
    cr = B.decode(v, zero_copy=True)
    blob = cr["parameters"]["blob"]
    assert isinstance(blob, memoryview) and bytes(blob) == d["parameters"]["blob"]
    assert is_pinned(np.frombuffer(blob, np.uint8).ctypes.data, len(blob))


def _rows(N, P, seed, shapes=((10, 10), (7,), None)):
    X = synth.clients_f32(seed, N, 0, P)
    out = []
    for i in range(N):
        r, layers, off = X[i], [], 0
        for shp in shapes:
            n = int(np.prod(shp)) if shp else P - off
            layers.append(r[off:off + n].reshape(shp) if shp else r[off:off + n])
            off += n
        out.append(layers)
    return out


def _same_outputs(a, b):
    return len(a) == len(b) and all(x.shape == y.shape and x.dtype == y.dtype and G.same_bits(x, y)
                                    for x, y in zip(a, b))


@pytest.mark.parametrize("case", ["plain", "scored", "short_scores", "f64_weight_late", "f64_layer_late",
                                  "ragged_beyond_scores", "int_layers", "one_row"])
def test_aggregate_decoded_equals_materialised(dev, case):
    """The overlapped decode+fold entry gives exactly what aggregate_layers gives
    on the materialised lists, including every fallback."""
    from fedlesscan_amd import engine
    N, P = 13, 2200
    rows = _rows(N, P, 31)
    w = list(synth.cardinalities(31, N))
    sc = [(r + 1) / 11 for r in synth.round_ids(31, N, 10, 2)]
    scores = None
    if case == "scored":
        scores = sc
    elif case == "short_scores":
        scores = sc[:5]
    elif case == "f64_weight_late":
        w[7] = np.float64(w[7])  # a strong scalar: numpy promotes the whole fold to float64
    elif case == "f64_layer_late":
        rows[6] = [x.astype(np.float64) for x in rows[6]]
    elif case == "ragged_beyond_scores":
        scores = sc[:4]
        rows[9] = rows[9][:2]  # never folded (zip truncation), only its weight counts
    elif case == "int_layers":
        rows = [[(x * 100).astype(np.int32) for x in r] for r in rows]
    elif case == "one_row":
        rows, w = rows[:1], w[:1]
    if case == "f64_layer_late":
        from fedlesscan_amd.aggregator.exceptions import InvalidParameterShapeError
        with pytest.raises(InvalidParameterShapeError):
            engine.aggregate_layers(rows, w, scores, device=dev)
        with pytest.raises(InvalidParameterShapeError):
            engine.aggregate_decoded(iter(list(zip(rows, w))), scores, device=dev)
        return
    exp = engine.aggregate_layers(rows, w, scores, device=dev)
    got = engine.aggregate_decoded(iter(list(zip(rows, w))), scores, device=dev)
    assert _same_outputs(got, exp)


# ---------------------------------------------------------------------------
# the native pipe (fa_ingest_*, csrc/ingest_pipe.cpp): worker-pool packs, an
# issuer thread per pipe, K chunk slots, the fold carried across them
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("chunk_rows", [1, 2, 5, 64])
@pytest.mark.parametrize("slots", [2, 3, 7])
@pytest.mark.parametrize("scored", [False, True])
def test_native_pipe_bit_exact(dev, chunk_rows, slots, scored):
    from fedlesscan_amd.ingest import NativeStreamingFold
    N, P = 37, 70001
    X = synth.clients_f32(61, N, 0, P)
    w = synth.cardinalities(61, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(61, N, 10, 2)] if scored else None
    ldx = (P + 63) // 64 * 64
    sf = NativeStreamingFold(P, dev, chunk_bytes=chunk_rows * ldx * 4, slots=slots)
    sf.acc.fill_(float("nan"))
    for i in range(N):
        r = X[i]
        # pieces that cross the 1 MiB copy-task boundary and tiny ones
        sf.add([r[:3].reshape(3), r[3:29903].reshape(100, 299), r[29903:]], w[i], None if sc is None else sc[i])
    got = sf.finish().cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert G.same_bits(got, exp)


def test_native_pipe_rounds_reuse_and_concurrency(dev):
    """A pipe serves round after round (the cache hands it back), two rounds in
    flight at once get two pipes, the divisor override (zip truncation) and a
    round whose rows fill the last slot exactly (finalize-only step)."""
    from fedlesscan_amd.ingest import NativeStreamingFold
    N, P = 12, 4099
    X = synth.clients_f32(62, N, 0, P)
    w = synth.cardinalities(62, N)
    ldx = (P + 63) // 64 * 64
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    for _ in range(3):
        a = NativeStreamingFold(P, dev, chunk_bytes=3 * ldx * 4, slots=2)  # 12 rows = 4 full slots
        b = NativeStreamingFold(P, dev, chunk_bytes=3 * ldx * 4, slots=2)
        assert a.pipe.value != b.pipe.value
        for i in range(N):
            a.add(X[i], w[i])
            b.add(X[N - 1 - i], w[N - 1 - i])
        assert G.same_bits(a.finish().cpu().numpy(), exp)
        got_b = b.finish(total=sum(w) + 5).cpu().numpy()
        exp_b = OL.fedavg_f32(X[::-1].copy(), np.array(w[::-1], np.float32), np.float32(sum(w) + 5))
        assert G.same_bits(got_b, exp_b)


def test_native_pipe_errors(dev):
    from fedlesscan_amd.aggregator.exceptions import InsufficientClientResults, InvalidParameterShapeError
    from fedlesscan_amd.ingest import NativeStreamingFold
    P = 1000
    sf = NativeStreamingFold(P, dev, chunk_bytes=1 << 20, slots=2)
    with pytest.raises(InvalidParameterShapeError):
        sf.add(np.zeros(999, np.float32), 1)
    with pytest.raises(InvalidParameterShapeError):  # a failed round is not reused
        sf.add(np.zeros(1000, np.float32), 1)
    sf = NativeStreamingFold(P, dev, chunk_bytes=1 << 20, slots=2)
    with pytest.raises(InvalidParameterShapeError):
        sf.add(np.zeros(1000, np.float64), 1)
    sf = NativeStreamingFold(P, dev, chunk_bytes=1 << 20, slots=2)
    sf.add(np.ones(1000, np.float32), 2)
    with pytest.raises(InvalidParameterShapeError):  # scores on some rows only
        sf.add(np.ones(1000, np.float32), 2, 0.5)
    sf = NativeStreamingFold(P, dev, chunk_bytes=1 << 20, slots=2)
    with pytest.raises(InsufficientClientResults):
        sf.finish()
    # the next round on a fresh pipe works
    sf = NativeStreamingFold(P, dev, chunk_bytes=1 << 20, slots=2)
    sf.add(np.full(1000, 3, np.float32), 2)
    assert np.all(sf.finish().cpu().numpy() == 3)


def test_native_pipe_is_the_default_aggregate_route(dev):
    """FedAvgAggregator.aggregate on host NPZ blobs goes through the native
    pipe and stays bit-exact against the reference goldens."""
    from fedlesscan_amd import FedAvgAggregator
    from fedlesscan_amd.ingest import NativeStreamingFold
    from test_gpu_multigpu import _npz_results
    case = "f32_n60"
    m = G.manifest()[case]
    before = NativeStreamingFold.stats["rows"]
    out = FedAvgAggregator().aggregate(_npz_results(G.parameters(case), m["weights"]), None)[0]
    assert NativeStreamingFold.stats["rows"] - before == len(m["weights"])
    assert all(G.same_bits(a, b) for a, b in zip(out, G.expected(case, "aggregate")))


@pytest.mark.parametrize("expected", ["none", "exact", "high", "low"])
@pytest.mark.parametrize("chunk_rows", [1, 4, 16])
def test_native_pipe_chunk_ramps(dev, expected, chunk_rows):
    """The ramps (first chunks of 1, 2, 4, ... rows; with the row count
    announced, last chunks of at most half of what is left) change only where
    the chunks end: bit-exact whatever count is announced."""
    from fedlesscan_amd.ingest import NativeStreamingFold
    N, P = 29, 20011
    X = synth.clients_f32(63, N, 0, P)
    w = synth.cardinalities(63, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(63, N, 10, 2)]
    ldx = (P + 63) // 64 * 64
    exp_rows = {"none": 0, "exact": N, "high": N + 5, "low": N - 7}[expected]
    sf = NativeStreamingFold(P, dev, chunk_bytes=chunk_rows * ldx * 4, slots=3, expected_rows=exp_rows)
    for i in range(N):
        sf.add(X[i], w[i], sc[i])
    got = sf.finish().cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)), s=np.array(sc, np.float32))
    assert G.same_bits(got, exp)


def test_native_pipe_abandoned_round_then_reuse_raw_abi(dev):
    """Through the C-ABI: a round abandoned with a chunk half filled (no finish),
    then fa_ingest_begin on the SAME pipe: the abandoned rows are dropped, the
    new round is bit-exact (the Python class never reuses a failed pipe; the
    C-ABI contract allows it)."""
    import ctypes

    import torch

    from fedlesscan_amd import _lib
    L = _lib.load()
    N, P = 9, 5003
    X = synth.clients_f32(64, N, 0, P)
    w = synth.cardinalities(64, N)
    ldx = (P + 63) // 64 * 64
    h = ctypes.c_void_p()
    _lib.call("fa_ingest_create", ctypes.byref(h), P, 4 * ldx * 4, 3, dev.index)
    try:
        acc = torch.empty(P, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        junk = np.full(P, 1e6, np.float32)
        ptrs = (ctypes.c_void_p * 1)(junk.ctypes.data)
        size = (ctypes.c_int64 * 1)(junk.nbytes)
        _lib.check(L.fa_ingest_begin(h, acc.data_ptr(), st, 0), "begin")
        for _ in range(2):  # chunk 0 takes 1 row (sent), chunk 1 ramps to 2 rows: half filled
            _lib.check(L.fa_ingest_add(h, ptrs, size, 1, 5.0, 1.0, 0), "add junk")
        _lib.check(L.fa_ingest_begin(h, acc.data_ptr(), st, N), "begin after an abandoned round")
        for i in range(N):
            row = np.ascontiguousarray(X[i])
            _lib.check(L.fa_ingest_add(h, (ctypes.c_void_p * 1)(row.ctypes.data), (ctypes.c_int64 * 1)(row.nbytes),
                                       1, float(np.float32(w[i])), 1.0, 0), "add")
        _lib.check(L.fa_ingest_finish(h, float(np.float32(sum(w)))), "finish")
        got = acc.cpu().numpy()
    finally:
        L.fa_ingest_destroy(h)
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    assert G.same_bits(got, exp)
