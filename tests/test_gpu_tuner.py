"""The measured form choice (fa_set_autotune, csrc/fold_kernels.hpp Tuner).

The first call of a new shape runs every candidate kernel form on the
caller's data (an untimed launch, then a timed batch each); later calls run
the fastest once the events are in.  All forms compute the same bits, so:
every form the tuner can choose is checked bit for bit against the oracle
(the fold of fed_avg_aggregator.py:24-42 / stall_aware_aggregation.py:42-67)
through the bench library's per-form entry, on shapes covering narrow (LDS
forms), a few tiles per CU (every form), large (grid-stride forms), P % 4 /
P % 8 tails, a padded row pitch and one client; and the tuned product calls
themselves -- the exploring call and the calls after the decision -- are
bit-exact too.
"""
import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth
from oracle import oracle_lib as OL  # checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

F32_SHAPES = [  # (N, P, extra row pitch, scored)
    (1, 1003, 0, False),
    (3, 4099, 0, True),
    (17, 70001, 0, False),
    (33, 65536 * 4 + 5, 0, True),
    (64, 909123, 0, False),
    (300, 1048579, 0, True),
    (1024, 65536, 0, False),
    (10, 5000, 128, False),
    (7, 2_000_001, 0, False),
]
BF16_SHAPES = [(5, 3001, False), (129, 1_048_583, True), (200, 1_100_003, False)]


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def L():
    from fedlesscan_amd import _lib
    lib = _lib.load()
    prev = lib.fa_set_autotune(1)
    yield lib
    lib.fa_set_autotune(prev)


def _run_until_tuned(L, fold, form, max_calls=8):
    """Call fold() until fa_fold_form names a form; returns the outputs of every call."""
    outs = []
    for _ in range(max_calls):
        outs.append(fold())
        torch.cuda.synchronize()
        if form():
            break
    return outs


@pytest.mark.parametrize("N,P,pad,scored", F32_SHAPES)
def test_f32_every_form_and_the_tuned_calls_bit_exact(dev, L, N, P, pad, scored):
    from fedlesscan_amd import _lib
    B = _lib.load_bench()
    seed = 71 + N
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    ldx = (P + 63) // 64 * 64 + pad  # 16-B rows (the vector path, the one the tuner measures); P % 4 tails stay
    Xd = torch.zeros((N, ldx), dtype=torch.float32, device=dev)
    Xd[:, :P] = torch.from_numpy(X).to(dev)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = None if sc is None else torch.tensor(np.array(sc, np.float32), device=dev)
    sp = None if s is None else s.data_ptr()
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    for f in range(B.fa_num_f32_forms()):  # every form the policy or the tuner can run
        o = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
        _lib.check(B.fa_fedavg_f32_form(Xd.data_ptr(), N, P, ldx, a.data_ptr(), sp, div, o.data_ptr(), st, f),
                   "form", bench=True)
        assert G.same_bits(o.cpu().numpy(), exp), (B.fa_f32_form_name(f), N, P)

    def fold():
        o = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
        _lib.check(L.fa_fedavg_f32(Xd.data_ptr(), N, P, ldx, a.data_ptr(), sp, div, o.data_ptr(), st), "fold")
        return o

    form = lambda: L.fa_fold_form(1, N, P, ldx, 1 if scored else 0, st).decode()  # noqa: E731
    assert form() == B.fa_f32_pick_name(N, P, 0).decode()  # unseen: the policy's form
    outs = _run_until_tuned(L, fold, form)
    assert form(), f"{N} x {P}: no decision after {len(outs)} calls"
    outs.append(fold())  # the decided form
    for k, o in enumerate(outs):
        assert G.same_bits(o.cpu().numpy(), exp), (N, P, k)


@pytest.mark.parametrize("N,P,scored", BF16_SHAPES)
def test_bf16_every_form_and_the_tuned_calls_bit_exact(dev, L, N, P, scored):
    from fedlesscan_amd import _lib
    B = _lib.load_bench()
    seed = 91 + N
    Xb = synth.clients_bf16(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    ldx = (P + 7) // 8 * 8
    Xd = torch.zeros((N, ldx), dtype=torch.int16, device=dev)
    Xd[:, :P] = torch.from_numpy(Xb.view(np.int16)).to(dev)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = None if sc is None else torch.tensor(np.array(sc, np.float32), device=dev)
    sp = None if s is None else s.data_ptr()
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    ef, eb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)),
                            s=None if sc is None else np.array(sc, np.float32))

    def fresh():
        return (torch.full((P,), float("nan"), dtype=torch.float32, device=dev),
                torch.zeros((P,), dtype=torch.int16, device=dev))

    for f in range(B.fa_num_bf16_forms()):
        o, ob = fresh()
        _lib.check(B.fa_fedavg_bf16_form(Xd.data_ptr(), N, P, ldx, a.data_ptr(), sp, div, o.data_ptr(),
                                         ob.data_ptr(), st, f), "bf16 form", bench=True)
        assert G.same_bits(o.cpu().numpy(), ef), (B.fa_bf16_form_name(f), N, P)
        assert np.array_equal(ob.cpu().numpy().view(np.uint16), eb), (B.fa_bf16_form_name(f), N, P)

    def fold():
        o, ob = fresh()
        _lib.check(L.fa_fedavg_bf16(Xd.data_ptr(), N, P, ldx, a.data_ptr(), sp, div, o.data_ptr(), ob.data_ptr(),
                                    st), "fa_fedavg_bf16")
        return o, ob

    form = lambda: L.fa_fold_form(2, N, P, ldx, 1 if scored else 0, st).decode()  # noqa: E731
    outs = _run_until_tuned(L, fold, form)
    assert form(), f"bf16 {N} x {P}: no decision after {len(outs)} calls"
    outs.append(fold())
    for k, (o, ob) in enumerate(outs):
        assert G.same_bits(o.cpu().numpy(), ef), (N, P, k)
        assert np.array_equal(ob.cpu().numpy().view(np.uint16), eb), (N, P, k)


def test_hostf_and_engine_path_tuned(dev, L):
    """engine.fold_stacked (the drop-in's path, *_hostf entries) goes through the
    tuner too: repeated calls of one shape stay bit-exact while it measures."""
    from fedlesscan_amd import engine
    N, P = 48, 600_004  # rows 16-B aligned: the vector path the tuner measures
    X = synth.clients_f32(5, N, 0, P)
    w = synth.cardinalities(5, N)
    Xd = torch.from_numpy(X).to(dev)
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(8):
        got = engine.fold_stacked(Xd, w).cpu().numpy()
        assert G.same_bits(got, exp)
        if L.fa_fold_form(1, N, P, P, 0, st):
            break
    assert L.fa_fold_form(1, N, P, P, 0, st)


def test_tuner_off_runs_the_policy_form(dev, L):
    from fedlesscan_amd import _lib
    B = _lib.load_bench()
    st = torch.cuda.current_stream(dev).cuda_stream
    N, P = 37, 777_777
    prev = L.fa_set_autotune(0)
    try:
        assert L.fa_set_autotune(-1) == 0
        assert L.fa_fold_form(1, N, P, P, 0, st) == B.fa_f32_pick_name(N, P, 0)
        X = synth.clients_f32(6, N, 0, P)
        w = synth.cardinalities(6, N)
        from fedlesscan_amd import engine
        got = engine.fold_stacked(torch.from_numpy(X).to(dev), w).cpu().numpy()
        assert G.same_bits(got, OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w))))
        assert L.fa_fold_form(1, N, P, P, 0, st) == B.fa_f32_pick_name(N, P, 0)  # still not measured
    finally:
        L.fa_set_autotune(prev)
    assert L.fa_fold_form(9, N, P, P, 0, st) == b""  # unknown kind


@pytest.mark.parametrize("N,P,scored", [(1, 5, False), (33, 4099, True), (100, 67267, False), (257, 20011, True),
                                        (64, 300_001, False), (40, 1_200_003, True)])
def test_row_table_every_form_and_the_tuned_calls_bit_exact(dev, L, N, P, scored):
    """fa_fedavg_f32_ptrs_aligned (separately allocated 16-B aligned rows, the
    engine's fold_rows path): every form it can choose, and its tuned calls."""
    from fedlesscan_amd import _lib
    B = _lib.load_bench()
    X = synth.clients_f32(211 + N, N, 0, P)
    w = synth.cardinalities(211 + N, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(211, N, 10, 2)] if scored else None
    rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]  # caching allocator: 256-B aligned rows
    tab = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = None if sc is None else torch.tensor(np.array(sc, np.float32), device=dev)
    sp = None if s is None else s.data_ptr()
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    for f in range(B.fa_num_ptrs_forms()):
        o = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
        _lib.check(B.fa_fedavg_f32_ptrs_form(tab.data_ptr(), N, P, a.data_ptr(), sp, div, o.data_ptr(), st, f),
                   "ptrs form", bench=True)
        assert G.same_bits(o.cpu().numpy(), exp), (B.fa_ptrs_form_name(f), N, P)

    def fold():
        o = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
        _lib.check(L.fa_fedavg_f32_ptrs_aligned(tab.data_ptr(), N, P, a.data_ptr(), sp, div, o.data_ptr(), st),
                   "fa_fedavg_f32_ptrs_aligned")
        return o

    form = lambda: L.fa_fold_form(3, N, P, P, 1 if scored else 0, st).decode()  # noqa: E731
    outs = _run_until_tuned(L, fold, form)
    assert form(), f"rows {N} x {P}: no decision after {len(outs)} calls"
    outs.append(fold())
    for k, o in enumerate(outs):
        assert G.same_bits(o.cpu().numpy(), exp), (N, P, k)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_output_over_the_rows_is_not_measured(dev, L, dt):
    """out inside the stacked rows (an in-place fold into row 0): the measuring
    call's later launches would read what earlier ones wrote, so such a call
    takes the policy's single launch and is still exact."""
    from fedlesscan_amd import _lib
    N, P = 64, 300_032
    w = synth.cardinalities(301, N)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    if dt == "f32":
        X = synth.clients_f32(301, N, 0, P)
        exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
        Xd = torch.from_numpy(X).to(dev)
        _lib.check(L.fa_fedavg_f32(Xd.data_ptr(), N, P, P, a.data_ptr(), None, div, Xd.data_ptr(), st), "in place")
        got = Xd[0].cpu().numpy()
        assert G.same_bits(got, exp)
        assert L.fa_fold_form(1, N, P, P, 0, st) == _lib.load_bench().fa_f32_pick_name(N, P, 0)  # never measured
    else:
        Xb = synth.clients_bf16(301, N, 0, P)
        ef, eb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)))
        Xd = torch.from_numpy(Xb.view(np.int16)).to(dev)
        o = torch.empty(P, dtype=torch.float32, device=dev)
        _lib.check(L.fa_fedavg_bf16(Xd.data_ptr(), N, P, P, a.data_ptr(), None, div, o.data_ptr(), Xd.data_ptr(), st),
                   "bf16 copy in place")
        assert G.same_bits(o.cpu().numpy(), ef)
        assert np.array_equal(Xd[0].cpu().numpy().view(np.uint16), eb)


def test_fold_inside_a_graph_capture(dev, L):
    """A fold captured into a HIP graph (torch.cuda.graph) takes the policy's
    single launch: no events are recorded inside a capture, and replays of
    the graph are bit-exact."""
    from fedlesscan_amd import _lib
    N, P = 48, 640_000
    X = synth.clients_f32(401, N, 0, P)
    w = synth.cardinalities(401, N)
    Xd = torch.from_numpy(X).to(dev)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    out = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            _lib.check(L.fa_fedavg_f32(Xd.data_ptr(), N, P, P, a.data_ptr(), None, div, out.data_ptr(),
                                       torch.cuda.current_stream(dev).cuda_stream), "captured fold")
    torch.cuda.current_stream(dev).wait_stream(s)
    assert L.fa_fold_form(1, N, P, P, 0, torch.cuda.current_stream(dev).cuda_stream) == \
        _lib.load_bench().fa_f32_pick_name(N, P, 0)  # nothing measured during the capture
    for _ in range(3):
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert G.same_bits(out.cpu().numpy(), exp)


@pytest.mark.parametrize("k", [0, 5])
def test_row_table_fold_into_one_of_its_rows(dev, L, k):
    """engine.fold_rows with out = rows[k]: the row table lives in
    device memory, so the library cannot see the alias, and the tuner's first
    call of a shape runs every candidate form into `out`.  fold_rows sees it
    on the host (RowSet.overlaps), folds into a fresh buffer and copies: the
    exploring call and the decided one are both bit-exact."""
    from fedlesscan_amd import engine
    N, P, seed = 12, 150_001 + 64 * k, 800 + k  # a shape of its own: its first call measures
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    for call in range(3):
        rows = [torch.from_numpy(X[i].copy()).to(dev) for i in range(N)]  # separate allocations: the table path
        rs = engine.RowSet(rows)
        assert rs.view is None and rs.overlaps(rows[k]) and not rs.overlaps(torch.empty(P, device=dev))
        got = engine.fold_rows(rs, w, out=rows[k])
        assert got.data_ptr() == rows[k].data_ptr()
        assert G.same_bits(rows[k].cpu().numpy(), exp), (k, call)
        torch.cuda.synchronize()
