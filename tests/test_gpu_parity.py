"""GPU parity: the HIP path (through the C-ABI) vs the pinned oracle / golden
vectors.  Contract: bit-exact for fp32/fp64/int outputs (NaN positions only,
payload not pinned); bf16 is defined as exact upcast + the fp32 fold, so it is
bit-exact against that definition too.  The one exception is the opt-in
split-client fold (exact=False), checked for determinism and normwise error."""
import ctypes

import numpy as np
import pytest

import golden_cases as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def lib():
    from fedlesscan_amd import _lib
    return _lib


def _bcheck(rc, what):
    """Status of a libfedavg_hip_bench.so call (variants, generator)."""
    from fedlesscan_amd import _lib
    _lib.check(rc, what, bench=True)


def _bits_equal(a, b):
    return G.same_bits(np.asarray(a), np.asarray(b))


def _sentinel(P, dev, dtype=None):
    """Output buffer pre-filled with NaN so an element the kernel never writes fails the test."""
    return torch.full((P,), float("nan"), dtype=dtype or torch.float32, device=dev)


# ---------------------------------------------------------------------------
# golden vectors through the drop-in strategy classes
# ---------------------------------------------------------------------------
def _npz_results(params, cards, b64=False):
    from fedlesscan_amd.common.models import (BinaryStringFormat, ClientResult, NpzWeightsSerializerConfig,
                                              SerializedParameters, WeightsSerializerConfig)
    from fedlesscan_amd.common.serialization import Base64StringConverter, NpzWeightsSerializer
    out = []
    for i, (p, c) in enumerate(zip(params, cards)):
        blob = NpzWeightsSerializer().serialize(p)
        fmt = BinaryStringFormat.NONE
        if b64 and i % 2 == 0:
            blob, fmt = Base64StringConverter.to_str(blob), BinaryStringFormat.BASE64
        out.append(ClientResult(parameters=SerializedParameters(
            blob=blob, serializer=WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig()),
            string_format=fmt), cardinality=c))
    return out


GOLDEN_LITERAL = [(c, p) for c, m in G.manifest().items() if not m.get("sampled")
                  for p in m["outputs"] if p in ("fedavg", "_aggregate", "stall")]


@pytest.mark.parametrize("case,prefix", GOLDEN_LITERAL)
def test_strategy_classes_match_golden(dev, case, prefix):
    from fedlesscan_amd import FedAvgAggregator, StallAwareAggregator
    from fedlesscan_amd.common.models import AggregationHyperParams
    m = G.manifest()[case]
    params = G.parameters(case)
    if prefix == "stall":
        out = StallAwareAggregator(m["current_round"], AggregationHyperParams(tolerance=2))._aggregate(
            G.feats(case), params, m["weights"])
    else:
        out = FedAvgAggregator()._aggregate(params, m["weights"])
    exp = G.expected(case, prefix)
    assert len(out) == len(exp)
    for a, b in zip(out, exp):
        assert a.shape == b.shape and a.dtype == b.dtype, (case, prefix, a.dtype, b.dtype)
        assert _bits_equal(a, b), (case, prefix)


def test_reference_fixture_aggregate_paths(dev):
    from fedlesscan_amd import FedAvgAggregator, StreamFedAvgAggregator, UnknownCardinalityError
    params = G.parameters("ref_fixture")
    res, _ = FedAvgAggregator().aggregate(_npz_results(params, [1, 2, 0], b64=True), None)
    assert all(_bits_equal(a, b) for a, b in zip(res, G.expected("ref_fixture", "aggregate_intcards")))
    bad = _npz_results(params, [-1, 2, 0], b64=True)
    with pytest.raises(UnknownCardinalityError):
        FedAvgAggregator().aggregate(bad, None)
    res, _ = FedAvgAggregator().aggregate(_npz_results(params, [-1, 2, 0], b64=True), None,
                                          default_cardinality=1.0)
    assert all(_bits_equal(a, b) for a, b in zip(res, G.expected("ref_fixture", "aggregate_default_card")))
    for cs in (1, 2, 10, 50):
        res, _ = StreamFedAvgAggregator(chunk_size=cs).aggregate(_npz_results(params, [1, 2, 0], True), None)
        assert all(_bits_equal(a, b) for a, b in zip(res, G.expected("ref_fixture", f"stream_c{cs}"))), cs


def test_n60_aggregate_and_stream_paths(dev):
    from fedlesscan_amd import (FedAvgAggregator, StallAwareAggregator, StreamFedAvgAggregator,
                                StreamStallAwareAggregator)
    from fedlesscan_amd.common.models import AggregationHyperParams
    case = "f32_n60"
    m = G.manifest()[case]
    params, w, feats, R = G.parameters(case), m["weights"], G.feats(case), m["current_round"]
    hp = AggregationHyperParams(tolerance=2)
    got = {
        "aggregate": FedAvgAggregator().aggregate(_npz_results(params, w), feats)[0],
        "aggregate_stall": StallAwareAggregator(R, hp).aggregate(_npz_results(params, w), feats)[0],
        "stream_c25": StreamFedAvgAggregator(25).aggregate(_npz_results(params, w), feats)[0],
        "stream_stall_c25": StreamStallAwareAggregator(R, hp, 25).aggregate(_npz_results(params, w), feats)[0],
    }
    for prefix, out in got.items():
        assert all(_bits_equal(a, b) for a, b in zip(out, G.expected(case, prefix))), prefix


def test_mnist_c1_sampled(dev):
    from fedlesscan_amd import FedAvgAggregator
    import hashlib
    case = "mnist_c1"
    m = G.manifest()[case]
    out = FedAvgAggregator()._aggregate(G.parameters(case), m["weights"])
    flat = np.concatenate([o.ravel() for o in out])
    assert hashlib.sha256(flat.tobytes()).hexdigest() == m["outputs"]["fedavg"]["flat_sha256"]


# ---------------------------------------------------------------------------
# kernels directly vs the C oracle: shapes, strides, alignment, variants
# ---------------------------------------------------------------------------
from oracle import oracle_lib as OL  # noqa: E402  (checker)
from fedlesscan_amd import synth  # noqa: E402


SHAPES = [(1, 1), (1, 4), (2, 3), (3, 5), (7, 1023), (16, 1024), (17, 1025), (33, 4099), (100, 65536),
          (129, 10007), (1000, 333)]


@pytest.mark.parametrize("N,P", SHAPES)
@pytest.mark.parametrize("scored", [False, True])
def test_fold_f32_shapes(dev, N, P, scored):
    from fedlesscan_amd import engine
    X = synth.clients_f32(1000 + N, N, 0, P)
    w = synth.cardinalities(1000 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(7, N, 10, 2)] if scored else None
    a = np.array(w, np.float32)
    s = None if sc is None else np.array(sc, np.float32)
    exp = OL.fedavg_f32(X, a, np.float32(sum(w)), s=s)
    got = engine.fold_stacked(torch.from_numpy(X).to(dev), w, sc, out=_sentinel(P, dev)).cpu().numpy()
    assert _bits_equal(got, exp)


@pytest.mark.parametrize("offset", [0, 1, 2, 3])
@pytest.mark.parametrize("pad", [0, 1, 5, 64])
def test_fold_f32_pitch_and_misalignment(dev, offset, pad):
    """Row pitch ldx > P and base offsets that break 16-B alignment (scalar path)."""
    from fedlesscan_amd import engine
    N, P = 9, 1030
    X = synth.clients_f32(5, N, 0, P)
    w = synth.cardinalities(5, N)
    big = torch.zeros((N, P + pad + offset), dtype=torch.float32, device=dev)
    big[:, offset:offset + P] = torch.from_numpy(X).to(dev)
    view = big[:, offset:offset + P]
    got = engine.fold_stacked(view, w, out=_sentinel(P, dev)).cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    assert _bits_equal(got, exp)


def test_all_variants_bit_identical(dev, lib):
    L = lib.load()
    B = lib.load_bench()
    N, P = 77, 50003
    X = torch.from_numpy(synth.clients_f32(8, N, 0, P)).to(dev)
    w = synth.cardinalities(8, N)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    s = torch.tensor([(r + 1) / 11 for r in synth.round_ids(8, N, 10, 2)], dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    for v in range(B.fa_num_variants()):
        for sp in (None, s):
            o = _sentinel(P, dev)
            _bcheck(B.fa_fedavg_f32_variant(X.data_ptr(), N, P, P, a.data_ptr(),
                                              None if sp is None else sp.data_ptr(),
                                              float(np.float32(sum(w))), o.data_ptr(), st, v), "variant")
            outs.append((v, sp is None, o.cpu().numpy()))
    base = {True: None, False: None}
    for v, plain, o in outs:
        if base[plain] is None:
            base[plain] = o
        assert _bits_equal(o, base[plain]), (v, plain)
    exp = OL.fedavg_f32(X.cpu().numpy(), np.array(w, np.float32), np.float32(sum(w)))
    assert _bits_equal(base[True], exp)


def test_chunked_fold_equals_batch(dev, lib):
    """fa_fold_f32 over row chunks (acc carried, divide at the end) == one batch fold."""
    L = lib.load()
    N, P = 50, 12345
    X = torch.from_numpy(synth.clients_f32(31, N, 0, P)).to(dev)
    w = synth.cardinalities(31, N)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    div = float(np.float32(sum(w)))
    acc = _sentinel(P, dev)
    bounds = [0, 1, 7, 20, 21, 49, 50]
    for k, (r0, r1) in enumerate(zip(bounds[:-1], bounds[1:])):
        last = r1 == N
        lib.check(L.fa_fold_f32(X[r0].data_ptr(), r1 - r0, P, P, a[r0:].data_ptr(), None,
                                None if k == 0 else acc.data_ptr(), div, int(last), acc.data_ptr(), st), "fold")
    exp = OL.fedavg_f32(X.cpu().numpy(), np.array(w, np.float32), np.float32(sum(w)))
    assert _bits_equal(acc.cpu().numpy(), exp)


@pytest.mark.parametrize("P", [4096, 16384, 16388, 30000, 32768])
@pytest.mark.parametrize("scored", [False, True])
def test_chunked_narrow_pipelined_fold(dev, lib, P, scored):
    """The narrowest picks (terms formed by the loaders, 4-6 chunks in flight)
    in their accumulate / finalize forms: chunks long enough for the deep
    pipeline (N = 700, 32-row chunks), acc carried, divide at the end."""
    L = lib.load()
    N = 700
    X = torch.from_numpy(synth.clients_f32(37 + P, N, 0, P)).to(dev)
    w = synth.cardinalities(37, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(37, N, 10, 2)]
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    s = torch.tensor(sc, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    div = float(np.float32(sum(w)))
    acc = _sentinel(P, dev)
    bounds = [0, 1, 250, 251, 699, 700]
    for k, (r0, r1) in enumerate(zip(bounds[:-1], bounds[1:])):
        lib.check(L.fa_fold_f32(X[r0].data_ptr(), r1 - r0, P, P, a[r0:].data_ptr(),
                                s[r0:].data_ptr() if scored else None,
                                None if k == 0 else acc.data_ptr(), div, int(r1 == N), acc.data_ptr(), st), "fold")
    exp = OL.fedavg_f32(X.cpu().numpy(), np.array(w, np.float32), np.float32(sum(w)),
                        s=np.array(sc, np.float32) if scored else None)
    assert _bits_equal(acc.cpu().numpy(), exp), (P, scored)


def test_ptr_rows_equal_stacked(dev):
    from fedlesscan_amd import engine
    N, P = 23, 7001
    X = synth.clients_f32(41, N, 0, P)
    w = synth.cardinalities(41, N)
    rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]
    # one misaligned row exercises the per-row scalar path
    holder = torch.zeros(P + 1, dtype=torch.float32, device=dev)
    holder[1:] = rows[3]
    rows[3] = holder[1:]
    sc = [(r + 1) / 11 for r in synth.round_ids(41, N, 10, 2)]
    for scores in (None, sc):
        got = engine.fold_rows(rows, w, scores).cpu().numpy()
        exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                            s=None if scores is None else np.array(scores, np.float32))
        assert _bits_equal(got, exp)


@pytest.mark.parametrize("N,P,pitch", [(2, 1, 1), (23, 7001, 7001), (23, 7001, 7003), (300, 67267, 67328),
                                       (64, 300_001, 300_001)])
@pytest.mark.parametrize("scored", [False, True])
@pytest.mark.parametrize("order", ["forward", "reversed"])
def test_view_rows_of_one_buffer(dev, N, P, pitch, scored, order):
    """Rows that are views of one buffer at a fixed pitch take the stacked fold
    (engine._equal_stride_view); reversed rows take the pointer-list fold.
    Both bit-equal to the oracle on the rows in the order given."""
    from fedlesscan_amd import engine
    X = synth.clients_f32(71 + N, N, 0, P)
    w = synth.cardinalities(71 + N, N)
    buf = torch.zeros(N * pitch + 3, dtype=torch.float32, device=dev)
    B = buf[3:].as_strided((N, P), (pitch, 1))  # odd storage offset when pitch is odd: unaligned rows
    B.copy_(torch.from_numpy(X))
    idx = list(range(N)) if order == "forward" else list(range(N))[::-1]
    rows = [B[i] for i in idx]
    assert (engine._equal_stride_view(rows, np.array([r.data_ptr() for r in rows]), P) is not None) == \
        (order == "forward")
    sc = [(r + 1) / 11 for r in synth.round_ids(72, N, 10, 2)] if scored else None
    got = engine.fold_rows(rows, [w[i] for i in idx], None if sc is None else [sc[i] for i in idx],
                           out=_sentinel(P, dev)).cpu().numpy()
    exp = OL.fedavg_f32(np.ascontiguousarray(X[idx]), np.array([w[i] for i in idx], np.float32),
                        np.float32(sum(w)), s=None if sc is None else np.array([sc[i] for i in idx], np.float32))
    assert _bits_equal(got, exp)


@pytest.mark.parametrize("N,P", [(1, 1), (3, 5), (23, 4099), (9, 1024 * 256 + 6), (5, 4 * 1024 * 256 + 3),
                                 (17, 4 * 1024 * 256 * 2 + 1)])
@pytest.mark.parametrize("scored", [False, True])
def test_aligned_ptr_rows(dev, N, P, scored):
    """fa_fedavg_f32_ptrs_aligned (every row 16-B aligned): both launch shapes
    (one block per 4 KiB tile, grid-stride 16 KiB tiles) and the column tail."""
    from fedlesscan_amd import engine
    X = synth.clients_f32(61 + N, N, 0, P)
    w = synth.cardinalities(61 + P, N)
    rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]
    assert all(r.data_ptr() % 16 == 0 for r in rows)
    sc = [(r + 1) / 11 for r in synth.round_ids(61, N, 10, 2)] if scored else None
    got = engine.fold_rows(rows, w, sc, out=_sentinel(P, dev)).cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert _bits_equal(got, exp)


@pytest.mark.parametrize("N,P", [(2, 3), (31, 16387), (33, 40003), (129, 67267), (300, 300_001), (1024, 4096)])
@pytest.mark.parametrize("scored", [False, True])
def test_rowset_lds_pointer_fold(dev, N, P, scored):
    """Separately allocated narrow rows take the LDS-staged fold with row bases
    read from the pointer table (every LDS pick: 16- and 32-quad tiles, the
    8-wave form at N >= 256); a RowSet built once refolds bit-exactly after
    its rows' contents change in place."""
    from fedlesscan_amd import engine
    X = synth.clients_f32(91 + N, N, 0, P)
    w = synth.cardinalities(91 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(91, N, 10, 2)] if scored else None
    rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]
    rs = engine.RowSet(rows)
    assert rs.view is None and rs.aligned
    s32 = None if sc is None else np.array(sc, np.float32)
    for rnd in range(2):
        got = engine.fold_rows(rs, w, sc, out=_sentinel(P, dev)).cpu().numpy()
        exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)), s=s32)
        assert _bits_equal(got, exp), rnd
        X = synth.clients_f32(191 + N, N, 0, P)  # next round: new contents, same tensors
        for i in range(N):
            rows[i].copy_(torch.from_numpy(X[i]))


@pytest.mark.parametrize("N,P", [(1, 5), (31, 16387), (33, 4099), (100, 67267), (257, 20011)])
def test_ptrs_loader_variants(dev, lib, N, P):
    """Every loader schedule / tile of the LDS pointer-table fold (tuning
    library): chunk edges (N % R), the last clamped block and the P % 4 tail
    block, plain and stall-aware, bit-exact vs the oracle."""
    B = lib.load_bench()
    X = synth.clients_f32(81 + N, N, 0, P)
    w = synth.cardinalities(81 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(81, N, 10, 2)]
    rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]
    tab = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    s = torch.tensor(sc, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)), s=np.array(sc, np.float32))
    assert B.fa_num_ptrs_variants() >= 8
    for v in range(B.fa_num_ptrs_variants()):
        for sp, e in ((None, exp), (s, exp_s)):
            o = _sentinel(P, dev)
            _bcheck(B.fa_fedavg_f32_ptrs_variant(tab.data_ptr(), N, P, a.data_ptr(),
                                                 None if sp is None else sp.data_ptr(), div, o.data_ptr(), st, v),
                    "ptrs variant")
            assert _bits_equal(o.cpu().numpy(), e), (B.fa_ptrs_variant_name(v), N, P, sp is not None)


@pytest.mark.parametrize("N,P", [(1, 7), (33, 4099), (257, 16387), (300, 67267), (70, 300_001)])
def test_ptrs_any_alignment(dev, lib, N, P):
    """Row tables whose rows are NOT 16-B aligned (X[i] of an unpadded [N, P]
    tensor with P % 4 != 0, shifted by one float): the product's
    fa_fedavg_f32_ptrs / RowSet path and every any-alignment pointer variant,
    plain and stall-aware, bit-exact vs the oracle."""
    from fedlesscan_amd import engine
    L, B = lib.load(), lib.load_bench()
    Xh = synth.clients_f32(520 + N, N, 0, P)
    buf = torch.zeros(N * P + 1, dtype=torch.float32, device=dev)
    X = buf[1:].view(N, P)
    X.copy_(torch.from_numpy(Xh).to(dev))
    rows = [X[i] for i in range(N)]
    tab = torch.tensor([r.data_ptr() for r in rows[::-1]], dtype=torch.int64, device=dev)  # reversed order
    w = synth.cardinalities(520 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(520 + N, N, 10, 2)]
    wr, scr = w[::-1], sc[::-1]
    a = torch.tensor(wr, dtype=torch.float32, device=dev)
    s = torch.tensor(scr, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    Xr = Xh[::-1].copy()
    exp = OL.fedavg_f32(Xr, np.array(wr, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(Xr, np.array(wr, np.float32), np.float32(sum(w)), s=np.array(scr, np.float32))
    vs = [v for v in range(B.fa_num_ptrs_variants())
          if B.fa_ptrs_variant_name(v).startswith((b"ptrs_dw", b"ptrs_rows_scalar", b"ptrs_generic"))]
    assert len(vs) >= 5
    for v in [None] + vs:
        for sp, e in ((None, exp), (s, exp_s)):
            o = _sentinel(P, dev)
            spp = None if sp is None else sp.data_ptr()
            if v is None:
                lib.check(L.fa_fedavg_f32_ptrs(tab.data_ptr(), N, P, a.data_ptr(), spp, div, o.data_ptr(), st), "ptrs")
            else:
                _bcheck(B.fa_fedavg_f32_ptrs_variant(tab.data_ptr(), N, P, a.data_ptr(), spp, div, o.data_ptr(), st,
                                                     v), "ptrs any-align variant")
            assert _bits_equal(o.cpu().numpy(), e), ("product" if v is None else B.fa_ptrs_variant_name(v), N, P,
                                                     sp is not None)
    rs = engine.RowSet(rows[::-1])
    assert rs.view is None and not rs.aligned
    assert _bits_equal(engine.fold_rows(rs, wr, scr, out=_sentinel(P, dev)).cpu().numpy(), exp_s)


@pytest.mark.parametrize("P", [67267, 32768, 40003, 131072, 200001, 81920])  # 4-wave 24/32/40-quad tiles, 2-wave 32
@pytest.mark.parametrize("N", [70, 257])
def test_lds_tile_picks(dev, lib, N, P):
    """Each column tile the auto policy picks for 32K-256K params: stacked and
    pointer-table folds, plain and stall-aware, and a two-part continued fold
    (acc carried across rows 0..32 | 33..N-1), all bit-exact vs the oracle."""
    from fedlesscan_amd import engine
    L = lib.load()
    X = synth.clients_f32(510 + N, N, 0, P)
    w = synth.cardinalities(510 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(510, N, 10, 2)]
    Xd = torch.from_numpy(X).to(dev)
    s32 = np.array(sc, np.float32)
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)), s=s32)
    assert _bits_equal(engine.fold_stacked(Xd, w, out=_sentinel(P, dev)).cpu().numpy(), exp)
    assert _bits_equal(engine.fold_stacked(Xd, w, sc, out=_sentinel(P, dev)).cpu().numpy(), exp_s)
    rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]
    assert _bits_equal(engine.fold_rows(rows, w, sc, out=_sentinel(P, dev)).cpu().numpy(), exp_s)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    div = float(np.float32(sum(w)))
    acc = _sentinel(P, dev)
    lib.check(L.fa_fold_f32(Xd.data_ptr(), 33, P, P, a.data_ptr(), None, None, div, 0, acc.data_ptr(), st), "f")
    lib.check(L.fa_fold_f32(Xd[33].data_ptr(), N - 33, P, P, a[33:].data_ptr(), None, acc.data_ptr(), div, 1,
                            acc.data_ptr(), st), "f")
    assert _bits_equal(acc.cpu().numpy(), exp)


@pytest.mark.parametrize("N,P", [(10, 582026), (47, 262147), (1, 300_000), (30, 1_000_003), (100, 582026),
                                 (48, 262147), (111, 700_001), (112, 582026), (64, 300_001),
                                 (10, 4 * 1024 * 1024 + 5), (23, 1024 * 1024 * 2 + 7),
                                 # the round-3 16 KiB plain-store tile pick (48+ clients, 0.7-1 tiles per CU)
                                 (48, 786_001), (64, 800_002), (100, 1_000_003), (130, 740_001)])
def test_few_client_tile_picks(dev, lib, N, P):
    """The few-client picks (a block per 4 KiB tile below one tile per CU; one
    lane per column at 48-111 clients below 3/4 of a tile per CU; a block per
    16 KiB tile under 24 clients above it) and their neighbours: plain,
    stall-aware and a two-part continued fold, bit-exact vs the oracle."""
    from fedlesscan_amd import engine
    L = lib.load()
    X = synth.clients_f32(530 + N, N, 0, P)
    w = synth.cardinalities(530 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(530, N, 10, 2)]
    ldx = (P + 63) // 64 * 64  # padded pitch: 16-B aligned rows take the vector picks
    Xd = torch.full((N, ldx), float("nan"), dtype=torch.float32, device=dev)[:, :P]
    Xd.copy_(torch.from_numpy(X))
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)), s=np.array(sc, np.float32))
    assert _bits_equal(engine.fold_stacked(Xd, w, out=_sentinel(P, dev)).cpu().numpy(), exp)
    assert _bits_equal(engine.fold_stacked(Xd, w, sc, out=_sentinel(P, dev)).cpu().numpy(), exp_s)
    Xu = torch.from_numpy(X).to(dev)  # unpadded (odd pitch when P % 4 != 0)
    assert _bits_equal(engine.fold_stacked(Xu, w, sc, out=_sentinel(P, dev)).cpu().numpy(), exp_s)
    if N > 1:
        h = N // 2
        a = torch.tensor(w, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        div = float(np.float32(sum(w)))
        acc = _sentinel(P, dev)
        lib.check(L.fa_fold_f32(Xd.data_ptr(), h, P, ldx, a.data_ptr(), None, None, div, 0, acc.data_ptr(), st),
                  "f")
        lib.check(L.fa_fold_f32(Xd[h].data_ptr(), N - h, P, ldx, a[h:].data_ptr(), None, acc.data_ptr(), div, 1,
                                acc.data_ptr(), st), "f")
        assert _bits_equal(acc.cpu().numpy(), exp)


def test_rowset_rejects_mixed_rows(dev):
    from fedlesscan_amd import InvalidParameterShapeError, engine
    with pytest.raises(InvalidParameterShapeError):
        engine.RowSet([torch.zeros(4, device=dev), torch.zeros(5, device=dev)])
    with pytest.raises(InvalidParameterShapeError):
        engine.RowSet([torch.zeros(4, device=dev), torch.zeros(4, device=dev, dtype=torch.float64)])
    rs = engine.RowSet([torch.zeros(4, device=dev), torch.zeros(4, device=dev)])
    with pytest.raises(InvalidParameterShapeError):
        engine.fold_rows(rs, [1, 2, 3])
    with pytest.raises(InvalidParameterShapeError):  # a non-contiguous row
        engine.RowSet([torch.zeros(4, device=dev), torch.zeros(8, device=dev)[::2]])
    with pytest.raises(InvalidParameterShapeError):  # a row on the host
        engine.RowSet([torch.zeros(4, device=dev), torch.zeros(4)])


@pytest.mark.parametrize("kind", ["views", "separate", "f64"])
def test_rowset_multidim_rows(dev, kind):
    """Rows need not be 1-D: X[i] of an [N, a, b] tensor (the equal-stride
    view), separately allocated [a, b] tensors (the pointer table) and float64
    rows (stacked first), each bit-equal to the oracle on the flattened rows."""
    from fedlesscan_amd import engine
    N, a, b = 37, 61, 101
    X = synth.clients_f32(601, N, 0, a * b)
    w = synth.cardinalities(602, N)
    if kind == "f64":
        X = X.astype(np.float64)
    X3 = torch.from_numpy(X.reshape(N, a, b)).to(dev)
    rows = [X3[i] for i in range(N)] if kind == "views" else [X3[i].clone() for i in range(N)]
    rs = engine.RowSet(rows)
    assert (rs.view is not None) == (kind == "views")
    got = engine.fold_rows(rs, w).cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w))) if kind != "f64" else \
        OL.fedavg_f64(X, np.array(w, np.float64), float(sum(w)))
    assert _bits_equal(got, exp)


@pytest.mark.parametrize("N,P", [(1, 8), (5, 9), (64, 8 * 1000 + 3), (256, 65536)])
@pytest.mark.parametrize("scored", [False, True])
def test_bf16_matches_definition(dev, N, P, scored):
    from fedlesscan_amd import engine
    Xb = synth.clients_bf16(60 + N, N, 0, P)
    w = synth.cardinalities(60 + N, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(60, N, 10, 2)] if scored else None
    exp, expb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)),
                               s=None if sc is None else np.array(sc, np.float32))
    Xd = torch.from_numpy(Xb.view(np.int16)).to(dev).view(torch.bfloat16)
    out, outb = engine.fold_stacked(Xd, w, sc, want_bf16=True, out=_sentinel(P, dev))
    assert _bits_equal(out.cpu().numpy(), exp)
    assert np.array_equal(outb.view(torch.int16).cpu().numpy().view(np.uint16), expb)


def test_bf16_variants_bit_identical(dev, lib):
    L = lib.load()
    B = lib.load_bench()
    N, P = 37, 8 * 3000 + 5
    Xb = synth.clients_bf16(71, N, 0, P)
    w = synth.cardinalities(71, N)
    exp, expb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)))
    Xd = torch.from_numpy(Xb.view(np.int16)).to(dev)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for v in range(B.fa_num_bf16_variants()):
        o = _sentinel(P, dev)
        ob = torch.full((P,), -1, dtype=torch.int16, device=dev)
        _bcheck(B.fa_fedavg_bf16_variant(Xd.data_ptr(), N, P, P, a.data_ptr(), None, float(np.float32(sum(w))),
                                           o.data_ptr(), ob.data_ptr(), st, v), "bf16 variant")
        assert _bits_equal(o.cpu().numpy(), exp), v
        assert np.array_equal(ob.cpu().numpy().view(np.uint16), expb), v


def test_f64_and_int_paths(dev):
    from fedlesscan_amd import engine
    X = np.stack([p[0] for p in G.parameters("f64_n40")])
    m = G.manifest()["f64_n40"]
    got = engine.fold_stacked(torch.from_numpy(X).to(dev), m["weights"]).cpu().numpy()
    assert _bits_equal(got, G.expected("f64_n40", "fedavg")[0])
    for case in ("int64_inputs", "int32_inputs"):
        m = G.manifest()[case]
        params = G.parameters(case)
        from fedlesscan_amd import FedAvgAggregator
        out = FedAvgAggregator()._aggregate(params, m["weights"])
        exp = G.expected(case, "fedavg")
        assert all(a.dtype == b.dtype and _bits_equal(a, b) for a, b in zip(out, exp)), case


def test_gpu_synth_matches_host(dev, lib):
    L = lib.load()
    B = lib.load_bench()
    st = torch.cuda.current_stream(dev).cuda_stream
    X = torch.empty((5, 3000), dtype=torch.float32, device=dev)
    _bcheck(B.fa_synth_f32(X.data_ptr(), 5, 2999, 3000, 77, 10, 123, st), "synth")
    exp = synth.clients_f32(77, 5, 123, 2999, row0=10)
    assert np.array_equal(X[:, :2999].cpu().numpy().view(np.uint32), exp.view(np.uint32))
    Xb = torch.empty((3, 1000), dtype=torch.int16, device=dev)
    _bcheck(B.fa_synth_bf16(Xb.data_ptr(), 3, 1000, 1000, 78, 0, 5, st), "synth_bf16")
    assert np.array_equal(Xb.cpu().numpy().view(np.uint16), synth.clients_bf16(78, 3, 5, 1000))


def test_host_factor_entries_reuse_slots(dev, lib):
    """fa_*_hostf: factors handed over in host memory.  More calls than the
    library's staging slots, queued without synchronising, with the host
    arrays overwritten right after each call, and client counts that make the
    slots grow: every result still bit-exact vs the oracle."""
    L = lib.load()
    st = torch.cuda.current_stream(dev).cuda_stream
    P = 4099
    Nmax = 9001  # with scores: 18002 floats > a slot's initial 16384
    X = torch.from_numpy(synth.clients_f32(17, Nmax, 0, P)).to(dev)
    Xh = X.cpu().numpy()
    Xb = torch.from_numpy(synth.clients_bf16(18, 40, 0, P).view(np.int16)).to(dev)
    rows = [X[i].clone() for i in range(64)]
    tab = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
    jobs = []
    for k in range(21):
        N = (3, 64, 40, 700, Nmax)[k % 5]
        w = synth.cardinalities(300 + k, N)
        sc = [(r + 1) / 11 for r in synth.round_ids(300 + k, N, 10, 2)] if k % 2 else None
        a = np.array(w, np.float32)
        s = None if sc is None else np.array(sc, np.float32)
        div = float(np.float32(sum(w)))
        sp = None if s is None else s.ctypes.data
        kind = ("stacked", "ptrs", "bf16")[k % 3] if N <= 64 else "stacked"
        if kind == "bf16" and N > 40:
            kind = "stacked"
        o = _sentinel(P, dev)
        if kind == "stacked":
            lib.check(L.fa_fedavg_f32_hostf(X.data_ptr(), N, P, P, a.ctypes.data, sp, div, o.data_ptr(), st), "hostf")
            exp = OL.fedavg_f32(Xh[:N], a, np.float32(sum(w)), s=s)
        elif kind == "ptrs":
            lib.check(L.fa_fedavg_f32_ptrs_hostf(tab.data_ptr(), N, P, a.ctypes.data, sp, div, k % 4 == 1,
                                               o.data_ptr(), st), "ptrs_hostf")
            exp = OL.fedavg_f32(Xh[:N], a, np.float32(sum(w)), s=s)
        else:
            lib.check(L.fa_fedavg_bf16_hostf(Xb.data_ptr(), N, P, P, a.ctypes.data, sp, div, o.data_ptr(), None, st),
                   "bf16_hostf")
            from oracle import fedavg_oracle as O
            exp, _ = O.fedavg_stacked_bf16(synth.clients_bf16(18, 40, 0, P)[:N], w, sc)
        a[:] = -7.0  # the library copied them: overwriting now must not matter
        if s is not None:
            s[:] = 3.0
        jobs.append((o, exp, kind, N))
    for o, exp, kind, N in jobs:
        assert _bits_equal(o.cpu().numpy(), np.asarray(exp, np.float32)), (kind, N)
    with pytest.raises(Exception):
        lib.check(L.fa_fedavg_f32_hostf(X.data_ptr(), 0, P, P, None, None, 1.0, X.data_ptr(), st), "hostf N=0")


def test_error_mapping(dev, lib):
    from fedlesscan_amd import FedAvgAggregator, InsufficientClientResults, InvalidParameterShapeError
    L = lib.load()
    X = torch.zeros((2, 8), device=dev)
    a = torch.ones(2, device=dev)
    with pytest.raises(InsufficientClientResults):
        lib.check(L.fa_fedavg_f32(X.data_ptr(), 0, 8, 8, a.data_ptr(), None, 1.0, X.data_ptr(), None), "x")
    with pytest.raises(InvalidParameterShapeError):
        lib.check(L.fa_fedavg_f32(X.data_ptr(), 2, 8, 4, a.data_ptr(), None, 1.0, X.data_ptr(), None), "x")
    with pytest.raises(ValueError):
        lib.check(L.fa_fedavg_f32(None, 2, 8, 8, a.data_ptr(), None, 1.0, X.data_ptr(), None), "x")
    with pytest.raises(InvalidParameterShapeError):
        FedAvgAggregator()._aggregate([[np.zeros(3, np.float32)], [np.zeros(4, np.float32)]], [1, 1])
    assert FedAvgAggregator()._aggregate([], []) == []


# ---------------------------------------------------------------------------
# BASELINE full sizes: exact on a column sample regenerated on the host
# ---------------------------------------------------------------------------
def _full_size_check(dev, lib, N, P, seed, dtype, scored, card_hi=600, block=1 << 20):
    """Generate the BASELINE-size workload in HBM, fold it on the GPU, then
    recompute EVERY output column on the host with the C oracle (regenerating
    the inputs block by block with the bit-identical host generator)."""
    from fedlesscan_amd import engine
    L = lib.load()
    B = lib.load_bench()
    st = torch.cuda.current_stream(dev).cuda_stream
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    X = torch.empty((N, P), dtype=tdt, device=dev)
    fn = B.fa_synth_f32 if dtype == "f32" else B.fa_synth_bf16
    lib.check(fn(X.data_ptr(), N, P, P, seed, 0, 0, st), "synth")
    w = synth.cardinalities(seed, N, 1, card_hi)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    out = engine.fold_stacked(X, w, sc, out=_sentinel(P, dev))
    got = out.cpu().numpy()
    del X, out
    torch.cuda.empty_cache()
    a = np.array(w, np.float32)
    s = None if sc is None else np.array(sc, np.float32)
    div = np.float32(sum(w))
    for c0 in range(0, P, block):
        nc = min(block, P - c0)
        if dtype == "f32":
            exp = OL.fedavg_f32(OL.synth_f32(seed, N, nc, col0=c0), a, div, s=s)
        else:
            exp = OL.fedavg_bf16(OL.synth_bf16(seed, N, nc, col0=c0), a, div, s=s)[0]
        assert _bits_equal(got[c0:c0 + nc], exp), (c0, nc)
    assert np.isfinite(got).all()


def test_config2_full_100x1M(dev, lib):
    from fedlesscan_amd import engine
    N, P, seed = 100, 1_000_000, 2
    X = OL.synth_f32(seed, N, P)
    w = synth.cardinalities(seed, N)
    got = engine.fold_stacked(torch.from_numpy(X).to(dev), w).cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    assert _bits_equal(got, exp)


def test_config3_full_size_1024x10M(dev, lib):
    _full_size_check(dev, lib, 1024, 10_000_000, 3, "f32", scored=False)


def test_config5_full_size_stall_512x25M(dev, lib):
    _full_size_check(dev, lib, 512, 25_000_000, 5, "f32", scored=True, card_hi=2000)


def test_config4_full_size_bf16_256x100M(dev, lib):
    # the whole config-4 model (256 x 100M bf16) on one GPU
    _full_size_check(dev, lib, 256, 100_000_000, 4, "bf16", scored=False)


@pytest.mark.parametrize("N,P,scored", [(256, 12_500_000, False),   # an 8-GPU rank's C4 bucket
                                        (256, 3_125_000, True),     # its round slot (4 rounds): 4 octets per lane
                                        (128, 4_000_011, False),    # same pick, P % 8 tail
                                        (256, 2_944_003, True),     # the pick's lower edge
                                        (256, 5_599_997, False)])   # its upper edge
def test_config4_rank_bucket_and_slots_bf16(dev, lib, N, P, scored):
    _full_size_check(dev, lib, N, P, 40 + N, "bf16", scored=scored)


@pytest.mark.parametrize("chunk_rows", [1, 3, 7, 64])
@pytest.mark.parametrize("scored", [False, True])
def test_streaming_fold_equals_batch(dev, chunk_rows, scored):
    from fedlesscan_amd.ingest import StreamingFold
    N, P = 29, 3001
    X = synth.clients_f32(91, N, 0, P)
    w = synth.cardinalities(91, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(91, N, 10, 2)] if scored else None
    sf = StreamingFold(P, chunk_rows=chunk_rows, device=dev)
    sf.acc.fill_(float("nan"))
    for i in range(N):
        # rows arrive as layer lists, like decoded NPZ members
        sf.add([X[i, :1000].reshape(10, 100), X[i, 1000:]], w[i], None if sc is None else sc[i])
    got = sf.finish().cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert _bits_equal(got, exp)


def test_sharded_aggregator_single_rank(dev):
    from fedlesscan_amd.sharding import ShardedAggregator
    N, P = 11, 5000
    X = synth.clients_f32(93, N, 0, P)
    w = synth.cardinalities(93, N)
    out = ShardedAggregator().aggregate(torch.from_numpy(X).to(dev), w)
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    assert _bits_equal(out.cpu().numpy(), exp)


TAIL_P = [1, 2, 3, 5, 1023, 1025, 1026, 1027, 2049, 4097, 8195, 4 * 1024 * 3 + 1, 4 * 2048 + 2, 40003]


@pytest.mark.parametrize("P", TAIL_P)
def test_every_variant_writes_every_column(dev, lib, P):
    """Column tails (P % 4 != 0) and partial last blocks for every fp32 variant,
    folded from scratch and as a continued chunked fold."""
    L = lib.load()
    B = lib.load_bench()
    N = 6
    X = torch.from_numpy(synth.clients_f32(300 + P, N, 0, P)).to(dev)
    w = synth.cardinalities(300 + P, N)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    exp = OL.fedavg_f32(X.cpu().numpy(), np.array(w, np.float32), np.float32(sum(w)))
    for v in range(B.fa_num_variants()):
        o = _sentinel(P, dev)
        _bcheck(B.fa_fedavg_f32_variant(X.data_ptr(), N, P, P, a.data_ptr(), None, div, o.data_ptr(), st, v),
                  "variant")
        assert _bits_equal(o.cpu().numpy(), exp), (v, P)
    acc = _sentinel(P, dev)
    lib.check(L.fa_fold_f32(X.data_ptr(), 2, P, P, a.data_ptr(), None, None, div, 0, acc.data_ptr(), st), "f")
    lib.check(L.fa_fold_f32(X[2].data_ptr(), N - 2, P, P, a[2:].data_ptr(), None, acc.data_ptr(), div, 1,
                            acc.data_ptr(), st), "f")
    assert _bits_equal(acc.cpu().numpy(), exp), P


@pytest.mark.parametrize("P", [1, 7, 9, 15, 2049, 2055, 8 * 256 * 2 + 3, 8 * 256 * 4 + 7, 65541])
def test_every_bf16_variant_writes_every_column(dev, lib, P):
    L = lib.load()
    B = lib.load_bench()
    N = 5
    Xb = synth.clients_bf16(400 + P, N, 0, P)
    w = synth.cardinalities(400 + P, N)
    exp, expb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)))
    Xd = torch.from_numpy(Xb.view(np.int16)).to(dev)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for v in range(B.fa_num_bf16_variants()):
        o = _sentinel(P, dev)
        ob = torch.full((P,), -1, dtype=torch.int16, device=dev)
        _bcheck(B.fa_fedavg_bf16_variant(Xd.data_ptr(), N, P, P, a.data_ptr(), None, float(np.float32(sum(w))),
                                           o.data_ptr(), ob.data_ptr(), st, v), "bf16 variant")
        assert _bits_equal(o.cpu().numpy(), exp), (v, P)
        assert np.array_equal(ob.cpu().numpy().view(np.uint16), expb), (v, P)


@pytest.mark.parametrize("strategy_name", ["fedlesscan", "fedavg"])
def test_config1_mock_aggregator_on_gpu(dev, strategy_name):
    """BASELINE config 1 end to end (store -> MockAggregator -> HIP fold -> NPZ
    -> parameter store), bit-exact against the reference-generated golden."""
    from test_host import config1_round
    res, shapes, sha, exp = config1_round(strategy_name)
    assert res.new_round_id == 11 and res.num_clients == 10
    assert [list(s) for s in shapes] == exp["shapes"]
    assert sha == exp["flat_sha256"]


@pytest.mark.parametrize("N,P,offset", [(1, 1, 0), (3, 7, 0), (40, 1001, 0), (17, 4097, 0), (9, 1000, 1)])
@pytest.mark.parametrize("scored", [False, True])
def test_f64_shapes_and_tails(dev, N, P, offset, scored):
    from fedlesscan_amd import engine
    X = synth.clients_f32(500 + P, N, 0, P).astype(np.float64) * (1.0 + 1.0 / 3.0)
    w = synth.cardinalities(500 + N, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(5, N, 10, 2)] if scored else None
    big = torch.zeros((N, P + offset), dtype=torch.float64, device=dev)
    big[:, offset:] = torch.from_numpy(X).to(dev)
    got = engine.fold_stacked(big[:, offset:], w, sc, out=_sentinel(P, dev, torch.float64)).cpu().numpy()
    exp = OL.fedavg_f64(X, np.array(w, np.float64), float(sum(w)),
                        s=None if sc is None else np.array(sc, np.float64))
    assert _bits_equal(got, exp)


@pytest.mark.parametrize("P", [1, 5, 4096, 10001])
@pytest.mark.parametrize("scored", [False, True])
def test_accumulate_finalize_equals_batch(dev, lib, P, scored):
    L = lib.load()
    N = 13
    X = synth.clients_f32(600 + P, N, 0, P)
    w = synth.cardinalities(600 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(600, N, 10, 2)] if scored else [1.0] * N
    Xd = torch.from_numpy(X).to(dev)
    acc = _sentinel(P, dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for i in range(N):
        lib.check(L.fa_accumulate_f32(acc.data_ptr(), Xd[i].data_ptr(), float(np.float32(w[i])),
                                      float(np.float32(sc[i])), int(i == 0), P, st), "acc")
    out = _sentinel(P, dev)
    lib.check(L.fa_finalize_f32(acc.data_ptr(), float(np.float32(sum(w))), out.data_ptr(), P, st), "fin")
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=np.array(sc, np.float32) if scored else None)
    assert _bits_equal(out.cpu().numpy(), exp)


def _lds_variants(B):
    return [v for v in range(B.fa_num_variants())
            if B.fa_variant_name(v).startswith((b"lds", b"ring", b"qf_", b"o0", b"o1", b"o2", b"dw_", b"scalar", b"pm_"))]


@pytest.mark.parametrize("N", [1, 2, 63, 64, 65, 127, 128, 129, 257, 300])
@pytest.mark.parametrize("P", [1, 3, 4, 255, 257, 4099, 16388])
def test_lds_variants_chunk_and_tile_edges(dev, lib, N, P):
    """The LDS-staged fold across its chunk (R rows) and tile (TQ quads)
    boundaries and the partial tail quad: plain, stall-aware, and a chunked
    continuation (acc carried, divide at the end), all bit-exact vs the oracle."""
    L = lib.load()
    B = lib.load_bench()
    X = torch.from_numpy(synth.clients_f32(700 + N, N, 0, P)).to(dev)
    w = synth.cardinalities(700 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(700 + N, N, 10, 2)]
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    s = torch.tensor(sc, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    Xh = X.cpu().numpy()
    exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)), s=np.array(sc, np.float32))
    variants = _lds_variants(B)
    assert len(variants) >= 4
    for v in variants:
        for sp, e in ((None, exp), (s, exp_s)):
            o = _sentinel(P, dev)
            _bcheck(B.fa_fedavg_f32_variant(X.data_ptr(), N, P, P, a.data_ptr(),
                                              None if sp is None else sp.data_ptr(), div, o.data_ptr(), st, v),
                      "lds variant")
            assert _bits_equal(o.cpu().numpy(), e), (B.fa_variant_name(v), N, P, sp is not None)


@pytest.mark.parametrize("N,P,pitch,off", [(1, 5, 5, 1), (33, 4099, 4099, 0), (70, 16387, 16390, 3),
                                           (257, 67267, 67267, 0), (100, 582026, 582027, 1), (31, 3, 7, 2)])
def test_any_alignment_variants(dev, lib, N, P, pitch, off):
    """The 4-byte-load LDS folds (and the scalar fold) on rows that are not
    16-B aligned: odd pitches and a base offset of 1-3 floats, plain and
    stall-aware, bit-exact vs the oracle; the product fold on the same layout."""
    L, B = lib.load(), lib.load_bench()
    Xh = synth.clients_f32(410 + N, N, 0, P)
    buf = torch.zeros(N * pitch + off + 4, dtype=torch.float32, device=dev)
    view = buf[off:off + N * pitch].view(N, pitch)[:, :P]
    view.copy_(torch.from_numpy(Xh).to(dev))
    w = synth.cardinalities(410 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(410 + N, N, 10, 2)]
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    s = torch.tensor(sc, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)), s=np.array(sc, np.float32))
    vs = [v for v in range(B.fa_num_variants()) if B.fa_variant_name(v).startswith((b"dw_", b"scalar", b"pm_dw_"))]
    assert len(vs) >= 6
    for v in [None] + vs:
        for sp, e in ((None, exp), (s, exp_s)):
            o = torch.full((P + 1,), float("nan"), dtype=torch.float32, device=dev)[1:]  # 4-B offset output
            spp = None if sp is None else sp.data_ptr()
            if v is None:
                lib.check(L.fa_fedavg_f32(view.data_ptr(), N, P, pitch, a.data_ptr(), spp, div, o.data_ptr(), st),
                          "auto")
            else:
                _bcheck(B.fa_fedavg_f32_variant(view.data_ptr(), N, P, pitch, a.data_ptr(), spp, div, o.data_ptr(),
                                                st, v), "any-align variant")
            name = "auto" if v is None else B.fa_variant_name(v)
            assert _bits_equal(o.cpu().numpy(), e), (name, N, P, pitch, off, sp is not None)


@pytest.mark.parametrize("N,P,pad", [(9, 1030, 2), (300, 65537, 63), (5, 300001, 3), (257, 2_100_003, 61),
                                     (260, 300_000, 0)])
@pytest.mark.parametrize("scored", [False, True])
def test_auto_picks_with_row_pitch(dev, lib, N, P, pad, scored):
    """Every kernel the auto policy picks (LDS-staged 4/8 waves, grid-stride),
    on a 16-B aligned row pitch ldx > P, with the P % 4 tail columns."""
    from fedlesscan_amd import engine
    ldx = P + pad + (-(P + pad)) % 4
    Xh = synth.clients_f32(900 + N, N, 0, P)
    big = torch.zeros((N, ldx), dtype=torch.float32, device=dev)
    big[:, :P] = torch.from_numpy(Xh).to(dev)
    big[:, P:] = float("nan")  # the pitch padding must never be read
    w = synth.cardinalities(900 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(900 + N, N, 10, 2)] if scored else None
    got = engine.fold_stacked(big[:, :P], w, sc, out=_sentinel(P, dev)).cpu().numpy()
    exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert _bits_equal(got, exp)


@pytest.mark.parametrize("N,P", [(300, 10007), (1024, 67267)])
def test_auto_fold_narrow_models(dev, lib, N, P):
    """Narrow-model shapes through the default entry point and a 3-way chunked
    continuation (the streaming-ingest call pattern)."""
    L = lib.load()
    X = torch.from_numpy(synth.clients_f32(800 + N, N, 0, P)).to(dev)
    w = synth.cardinalities(800 + P, N)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    exp = OL.fedavg_f32(X.cpu().numpy(), np.array(w, np.float32), np.float32(sum(w)))
    o = _sentinel(P, dev)
    lib.check(L.fa_fedavg_f32(X.data_ptr(), N, P, P, a.data_ptr(), None, div, o.data_ptr(), st), "auto")
    assert _bits_equal(o.cpu().numpy(), exp)
    acc = _sentinel(P, dev)
    cuts = [0, N // 3, N // 3 + 1, N]
    for k, (r0, r1) in enumerate(zip(cuts[:-1], cuts[1:])):
        lib.check(L.fa_fold_f32(X[r0].data_ptr(), r1 - r0, P, P, a[r0:].data_ptr(), None,
                                None if k == 0 else acc.data_ptr(), div, int(r1 == N), acc.data_ptr(), st), "f")
    assert _bits_equal(acc.cpu().numpy(), exp)


@pytest.mark.parametrize("case,prefix", [("f32_small", "fedavg"), ("f32_small", "stall"), ("f32_n60", "fedavg"),
                                         ("n1", "fedavg"), ("f64_n40", "fedavg"), ("specials", "fedavg")])
def test_device_tensor_inputs_match_golden(dev, case, prefix):
    """Layers already on the GPU (a device-resident simulation): fp32 goes through
    the pointer-list fold with no stacking copy; other dtypes are stacked."""
    from fedlesscan_amd import engine
    m = G.manifest()[case]
    params = [[torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in p] for p in G.parameters(case)]
    scores = None
    if prefix == "stall":
        scores = [(f["round_id"] + 1) / (m["current_round"] + 1) for f in G.feats(case)]
    out = engine.aggregate_layers(params, m["weights"], scores)
    exp = G.expected(case, prefix)
    assert len(out) == len(exp)
    for a, b in zip(out, exp):
        assert a.is_cuda and tuple(a.shape) == b.shape
        assert _bits_equal(a.cpu().numpy(), b), (case, prefix)


# ---------------------------------------------------------------------------
# opt-in split-client fold: deterministic, NOT bit-exact (different association)
# ---------------------------------------------------------------------------
def _normwise(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b.astype(np.float64))) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("N,P", [(1, 1), (3, 7), (2, 64), (33, 4099), (100, 10001), (1000, 333), (1024, 67267),
                                 (40, 65)])
@pytest.mark.parametrize("scored", [False, True])
def test_splitn_deterministic_and_close(dev, lib, N, P, scored):
    from fedlesscan_amd import engine
    Xh = synth.clients_f32(950 + N, N, 0, P)
    w = synth.cardinalities(950 + P, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(950 + N, N, 10, 2)] if scored else None
    X = torch.from_numpy(Xh).to(dev)
    o1 = engine.fold_stacked(X, w, sc, out=_sentinel(P, dev), exact=False).cpu().numpy()
    o2 = engine.fold_stacked(X, w, sc, out=_sentinel(P, dev), exact=False).cpu().numpy()
    assert _bits_equal(o1, o2)  # deterministic: a fixed tree, no atomics
    a = np.array(w, np.float32)
    s = None if sc is None else np.array(sc, np.float32)
    ref = OL.fedavg_f32(Xh, a, np.float32(sum(w)), s=s)  # the reference's left fold
    t = Xh.astype(np.float64) * a.astype(np.float64)[:, None]
    if s is not None:
        t *= s.astype(np.float64)[:, None]
    exact = t.sum(axis=0) / float(np.float32(sum(w)))  # fp64 sum of the fp32 products
    # tolerance: a few fp32 ulps of the accumulated magnitude (N adds of each association)
    tol = 4e-7 * max(1.0, np.log2(N) + 1)
    assert _normwise(o1, exact) <= tol, (_normwise(o1, exact), tol)
    assert _normwise(o1, ref) <= 2 * tol
    assert np.isfinite(o1).all()


def test_splitn_rejects_unaligned(dev, lib):
    L = lib.load()
    X = torch.zeros((4, 66), dtype=torch.float32, device=dev)
    a = torch.ones(4, dtype=torch.float32, device=dev)
    o = torch.zeros(64, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    # misaligned base and a row pitch that is not a multiple of 4 floats: refused at the C-ABI
    assert L.fa_fedavg_f32_splitn(X.data_ptr() + 4, 4, 64, 66, a.data_ptr(), None, 4.0, o.data_ptr(), st) == \
        lib.FA_ERR_ARG
    assert L.fa_fedavg_f32_splitn(X.data_ptr(), 4, 64, 66, a.data_ptr(), None, 4.0, o.data_ptr(), st) == \
        lib.FA_ERR_ARG
    # engine.fold_stacked(exact=False) takes the exact fold for such layouts instead
    from fedlesscan_amd import engine
    Xh = synth.clients_f32(3, 4, 0, 64)
    big = torch.zeros((4, 66), dtype=torch.float32, device=dev)
    big[:, 1:65] = torch.from_numpy(Xh).to(dev)
    got = engine.fold_stacked(big[:, 1:65], [1, 2, 3, 4], exact=False).cpu().numpy()
    assert _bits_equal(got, OL.fedavg_f32(Xh, np.array([1, 2, 3, 4], np.float32), np.float32(10)))


@pytest.mark.parametrize("scored", [False, True])
def test_empty_and_scalar_layers(dev, scored):
    """Layers with zero elements and 0-d layers next to ordinary ones, through
    the drop-in classes, against the oracle's literal numpy fold."""
    from oracle import fedavg_oracle as O
    from fedlesscan_amd import FedAvgAggregator, StallAwareAggregator
    from fedlesscan_amd.common.models import AggregationHyperParams
    N = 5
    rng = np.random.default_rng(3)
    params = [[rng.standard_normal((3, 4)).astype(np.float32), np.zeros((0, 5), np.float32),
               np.float32(rng.standard_normal()).reshape(()), rng.standard_normal(7).astype(np.float32)]
              for _ in range(N)]
    w = [3, 1, 4, 1, 5]
    if scored:
        feats = [{"round_id": r} for r in (8, 9, 10, 10, 9)]
        got = StallAwareAggregator(10, AggregationHyperParams(tolerance=2))._aggregate(feats, params, w)
        exp = O.stall_aware_literal(feats, 10, params, w)
    else:
        got = FedAvgAggregator()._aggregate(params, w)
        exp = O.fedavg_literal(params, w)
    assert [g.shape for g in got] == [e.shape for e in exp]
    for g, e in zip(got, exp):
        assert g.dtype == e.dtype and _bits_equal(g, e)


@pytest.mark.parametrize("N,P", [(64, 4099), (300, 300_001)])
def test_fold_captures_into_hip_graph(dev, lib, N, P):
    """The C-ABI enqueues only (no allocation, no synchronisation), so a fold
    captures into a HIP graph and replays bit-exactly on new inputs."""
    L = lib.load()
    X = torch.from_numpy(synth.clients_f32(71, N, 0, P)).to(dev)
    w = synth.cardinalities(71, N)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    out = _sentinel(P, dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rc = L.fa_fedavg_f32(X.data_ptr(), N, P, P, a.data_ptr(), None, div, out.data_ptr(), s.cuda_stream)
    assert rc == 0, lib.last_error()
    for seed in (72, 73):
        X.copy_(torch.from_numpy(synth.clients_f32(seed, N, 0, P)))
        g.replay()
        torch.cuda.synchronize()
        exp = OL.fedavg_f32(X.cpu().numpy(), np.array(w, np.float32), np.float32(sum(w)))
        assert _bits_equal(out.cpu().numpy(), exp)


def test_host_factor_entries_refuse_capture_fill_is_captured_by_value(dev, lib):
    """ABI 6: a _hostf entry on a capturing stream is an argument error (a
    graph would have to own the staged copy), not a launch; fa_factors_fill
    writes a, then s, into memory the graph owns by kernels that carry the
    values, so the replays fold with the captured factors after the caller's
    host arrays changed (the stall-aware fold, bit-exact)."""
    L = lib.load()
    N, P = 300, 4099
    X = torch.from_numpy(synth.clients_f32(81, N, 0, P)).to(dev)
    w = np.array(synth.cardinalities(81, N), np.float32)
    sc = np.linspace(0.25, 1.0, N, dtype=np.float32)
    w0, sc0 = w.copy(), sc.copy()
    div = float(np.float32(w.sum(dtype=np.float64)))
    out = _sentinel(P, dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rc_h = L.fa_fedavg_f32_hostf(X.data_ptr(), N, P, P, w.ctypes.data, None, div, out.data_ptr(), s.cuda_stream)
        msg = lib.last_error()
        buf = torch.empty(2 * N, dtype=torch.float32, device=dev)
        rc_f = L.fa_factors_fill(buf.data_ptr(), w.ctypes.data, sc.ctypes.data, N, s.cuda_stream)
        rc_k = L.fa_fedavg_f32(X.data_ptr(), N, P, P, buf.data_ptr(), buf.data_ptr() + 4 * N, div, out.data_ptr(),
                               s.cuda_stream)
    assert rc_h == lib.FA_ERR_ARG and "capture" in msg, msg
    assert rc_f == 0 and rc_k == 0, lib.last_error()
    w[:] = 0
    sc[:] = 0
    exp = OL.fedavg_f32(X.cpu().numpy(), w0, np.float32(div), sc0)
    for _ in range(3):
        out.fill_(float("nan"))
        buf.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), np.concatenate([w0, sc0]))
        assert _bits_equal(out.cpu().numpy(), exp)
    assert L.fa_factors_fill(None, w.ctypes.data, None, 4, s.cuda_stream) == lib.FA_ERR_ARG
    assert L.fa_factors_fill(None, None, None, 0, s.cuda_stream) == 0


def test_openfaas_entry_point_on_gpu(dev):
    """The FaaS entry point end to end on the HIP fold: request JSON in,
    response JSON out, the saved round+1 model bit-exact vs the oracle."""
    import json
    from oracle import fedavg_oracle as O
    from test_host import REF_REQUEST, _stores_with_round
    from fedlesscan_amd.common.serialization import NpzWeightsSerializer
    from fedlesscan_amd.functions import Event, make_openfaas_handler
    st, ps = _stores_with_round()
    ins = [(NpzWeightsSerializer().deserialize(r.parameters.blob), r.cardinality)
           for r in st.load_results_for_round("s", 3)[1]]
    resp = make_openfaas_handler(st, ps)(Event(json.dumps(REF_REQUEST)))
    assert resp["statusCode"] == 200, resp["body"]
    assert json.loads(resp["body"])["num_clients"] == 4
    got = NpzWeightsSerializer().deserialize(ps.load("s", 4).blob)
    exp = O.fedavg_literal([p for p, _ in ins], [c for _, c in ins])
    assert all(_bits_equal(g, e) for g, e in zip(got, exp))


@pytest.mark.parametrize("P", [4 * 1024 * 256 * 2 + 4096 * 3 + 3, 5_000_003])
def test_band_variants_multi_band(dev, lib, P):
    """Column-band launches (several kernels over contiguous column bands):
    every band boundary and the tail, plain, stall-aware and as a chunked
    continuation, bit-exact vs the oracle."""
    L = lib.load()
    B = lib.load_bench()
    N = 3
    X = torch.from_numpy(synth.clients_f32(81, N, 0, P)).to(dev)
    w = synth.cardinalities(81, N)
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    sc = [(r + 1) / 11 for r in synth.round_ids(81, N, 10, 2)]
    s = torch.tensor(sc, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    Xh = X.cpu().numpy()
    exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)))
    exp_s = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)), s=np.array(sc, np.float32))
    bands = [v for v in range(B.fa_num_variants()) if B.fa_variant_name(v).startswith(b"gsband")]
    assert bands
    for v in bands + [0]:
        for sp, e in ((None, exp), (s, exp_s)):
            o = _sentinel(P, dev)
            _bcheck(B.fa_fedavg_f32_variant(X.data_ptr(), N, P, P, a.data_ptr(),
                                              None if sp is None else sp.data_ptr(), div, o.data_ptr(), st, v), "v")
            assert _bits_equal(o.cpu().numpy(), e), (B.fa_variant_name(v), sp is not None)
    acc = _sentinel(P, dev)  # auto policy as a two-chunk continuation
    lib.check(L.fa_fold_f32(X.data_ptr(), 2, P, P, a.data_ptr(), None, None, div, 0, acc.data_ptr(), st), "f")
    lib.check(L.fa_fold_f32(X[2].data_ptr(), 1, P, P, a[2:].data_ptr(), None, acc.data_ptr(), div, 1,
                            acc.data_ptr(), st), "f")
    assert _bits_equal(acc.cpu().numpy(), exp)


@pytest.mark.parametrize("N", [1, 2, 7, 8, 9, 15, 16, 17, 33, 100])
@pytest.mark.parametrize("P", [4, 7, 260, 1028, 4 * 256 * 256 + 3, 300001, 800000])
def test_even_split_client_and_column_edges(dev, lib, N, P):
    """k_fold_f32_even (the even-split fold): client counts around its U rows
    in flight (row indices clamped, adds of rows past N skipped) and column
    ranges that end inside a lane's C quads (clamped quads never stored),
    stall-aware and plain, bit-exact against the C oracle."""
    B = lib.load_bench()
    names = [B.fa_variant_name(v).decode() for v in range(B.fa_num_variants())]
    evens = [v for v, n in enumerate(names) if n.startswith("even_")]
    assert len(evens) >= 8
    X = torch.from_numpy(synth.clients_f32(500 + N, N, 0, P)).to(dev)
    w = synth.cardinalities(500 + N, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(500 + N, N, 10, 2)]
    a = torch.tensor(w, dtype=torch.float32, device=dev)
    s = torch.tensor(sc, dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    Xh = X.cpu().numpy()
    for sp in (None, s):
        exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)),
                            s=None if sp is None else np.array(sc, np.float32))
        for v in evens:
            o = _sentinel(P, dev)
            _bcheck(B.fa_fedavg_f32_variant(X.data_ptr(), N, P, P, a.data_ptr(), None if sp is None else sp.data_ptr(),
                                            div, o.data_ptr(), st, v), "variant")
            assert _bits_equal(o.cpu().numpy(), exp), (names[v], N, P, sp is None)
