"""The one-launch exchange step (fa_fedavg_*_rounds, csrc/fold_kernels.hpp
step_tiles): every step form of the library and the product entry with its
per-round waits, bit for bit against the C oracle of fed_avg_aggregator.py:24-42
/ stall_aware_aggregation.py:42-67 (bf16: exact upcast + that fold).

Covered: the slot widths an 8-GPU C4 rank folds (sharding.overlap_layout(100M,
8, "bf16"): 256 clients, every column checked), a C3 rank's layout, eight
small rounds with an odd client count, a last round ending off an octet
boundary (its tail columns stored plainly beside write-through tiles),
stall-aware, each round's result
copied behind its wait on another stream the moment it is flagged, four
launches back to back on one state, and the argument checks.
"""
import numpy as np
import pytest

from fedlesscan_amd import synth
from fedlesscan_amd.sharding import overlap_layout
from oracle import oracle_lib as OL  # checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def libs():
    from fedlesscan_amd import _lib
    return _lib, _lib.load(), _lib.load_bench()


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def _one_launch_steps(dev, libs, X, N, W, lay, a, s, div, bf16):
    """Outputs of the one-launch step folds over lay's rounds (round k stall-
    aware when k is odd is not possible in one launch: all rounds plain when
    s is None, else all scored): {name: (f32 out, bf16 out or None)}.  The
    product launch repeats 4 times; each time, behind fa_rounds_wait(k) on a
    side stream, a copy of round k's columns is taken the moment the round is
    flagged complete -- the copies must hold the final bits."""
    import ctypes
    _lib, L, B = libs
    st = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    offs = (ctypes.c_int64 * (lay.rounds + 1))(*[lay.offset(k) for k in range(lay.rounds + 1)])
    sp = None if s is None else s.data_ptr()
    res = {}
    rb = ctypes.c_void_p()
    _lib.check(B.fa_bench_rounds_create(ctypes.byref(rb), dev.index), "rounds state", bench=True)
    for f in range(B.fa_num_step_forms()):
        name = B.fa_step_form_name(f).decode()
        if name.startswith("bf16") != bf16:
            continue
        o = torch.full((W,), float("nan"), dtype=torch.float32, device=dev)
        ob = torch.zeros((W,), dtype=torch.int16, device=dev) if bf16 else None
        _lib.check(B.fa_fedavg_rounds_form(rb, f, X.data_ptr(), N, W, a.data_ptr(), sp, div, o.data_ptr(),
                                           None if ob is None else ob.data_ptr(), lay.rounds, offs, st.cuda_stream),
                   "step form", bench=True)
        res[name] = (o.cpu().numpy(), None if ob is None else ob.cpu().numpy().view(np.uint16))
        if bf16:  # ABI 5: the bf16 result alone, no fp32 output
            ob2 = torch.zeros((W,), dtype=torch.int16, device=dev)
            _lib.check(B.fa_fedavg_rounds_form(rb, f, X.data_ptr(), N, W, a.data_ptr(), sp, div, None, ob2.data_ptr(),
                                               lay.rounds, offs, st.cuda_stream), "step form, bf16 only", bench=True)
            res[name + " bf16 only"] = (None, ob2.cpu().numpy().view(np.uint16))
    # the policy form publishing at system scope: sc0 sc1 tile stores (a peer
    # exchange's launches, sys 1) and round 5's per-block fence (sys 2)
    pol = L.fa_rounds_form(1 if bf16 else 0).decode()
    fpol = next(f for f in range(B.fa_num_step_forms()) if B.fa_step_form_name(f).decode() == pol)
    for sysm in (1, 2):
        _lib.check(B.fa_bench_rounds_set_sys(rb, sysm), "sys", bench=True)
        o = torch.full((W,), float("nan"), dtype=torch.float32, device=dev)
        ob = torch.zeros((W,), dtype=torch.int16, device=dev) if bf16 else None
        _lib.check(B.fa_fedavg_rounds_form(rb, fpol, X.data_ptr(), N, W, a.data_ptr(), sp, div,
                                           None if bf16 else o.data_ptr(), None if ob is None else ob.data_ptr(),
                                           lay.rounds, offs, st.cuda_stream), f"policy form sys {sysm}", bench=True)
        res[f"{pol} sys {sysm}"] = (None if bf16 else o.cpu().numpy(),
                                    None if ob is None else ob.cpu().numpy().view(np.uint16))
    _lib.check(B.fa_bench_rounds_destroy(rb), "destroy", bench=True)
    r = ctypes.c_void_p()
    _lib.check(L.fa_rounds_create(ctypes.byref(r), dev.index), "fa_rounds_create")
    o = torch.empty((W,), dtype=torch.float32, device=dev)
    ob = torch.empty((W,), dtype=torch.int16, device=dev) if bf16 else None
    for rep in range(4):
        o.fill_(float("nan"))
        if ob is not None:
            ob.fill_(-1)
        got = torch.full((W,), -1, dtype=torch.int16 if bf16 else torch.int32, device=dev)
        if bf16:  # reps 2-3 store the bf16 result alone (ABI 5: out_f32 NULL)
            rc = L.fa_fedavg_bf16_rounds(r, X.data_ptr(), N, W, a.data_ptr(), sp, div,
                                         o.data_ptr() if rep < 2 else None, ob.data_ptr(), lay.rounds, offs, None,
                                         st.cuda_stream)
        else:
            rc = L.fa_fedavg_f32_rounds(r, X.data_ptr(), N, W, a.data_ptr(), sp, div, o.data_ptr(), lay.rounds, offs,
                                        None, st.cuda_stream)
        _lib.check(rc, "rounds fold")
        src = ob if bf16 else o.view(torch.int32)
        for k in range(lay.rounds):
            _lib.check(L.fa_rounds_wait(r, k, side.cuda_stream), "rounds wait")
            with torch.cuda.stream(side):
                a0, a1 = lay.offset(k), lay.offset(k + 1)
                got[a0:a1].copy_(src[a0:a1])
        torch.cuda.synchronize()
        if bf16 and rep >= 2:
            assert np.isnan(o.cpu().numpy()).all()  # no fp32 store at all
            res[f"product rounds rep {rep}"] = (None, ob.cpu().numpy().view(np.uint16))
        else:
            res[f"product rounds rep {rep}"] = (o.cpu().numpy(), ob.cpu().numpy().view(np.uint16) if bf16 else None)
        g = got.cpu().numpy()
        res[f"copied behind the waits rep {rep}"] = ((None, g.view(np.uint16)) if bf16 else (g.view(np.float32), None))
    assert L.fa_rounds_timeouts(r) == 0 and L.fa_rounds_check(r) == 0
    _lib.check(L.fa_rounds_destroy(r), "destroy")
    return res


def test_bf16_one_launch_steps_at_the_c4_rank_slots(dev, libs):
    """One 8-GPU C4 rank: 256 clients x its four slots side by side (12.5M
    bf16 columns), stall-aware: every bf16 step form and the product entry
    with each round's result copied behind fa_rounds_wait on another stream,
    every column checked."""
    _lib, L, B = libs
    N, seed = 256, 44
    lay = overlap_layout(100_000_000, 8, "bf16")
    W = lay.local_width
    st = torch.cuda.current_stream(dev).cuda_stream
    X = torch.empty((N, W), dtype=torch.bfloat16, device=dev)
    _lib.check(B.fa_synth_bf16(X.data_ptr(), N, W, W, seed, 0, 0, st), "synth", bench=True)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = torch.tensor(np.array(sc, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    one = _one_launch_steps(dev, libs, X, N, W, lay, a, s, div, bf16=True)
    assert len(one) >= 10
    del X
    torch.cuda.empty_cache()
    an, sn = np.array(w, np.float32), np.array(sc, np.float32)
    for c0 in range(0, W, 1 << 20):
        nc = min(1 << 20, W - c0)
        ef, eb = OL.fedavg_bf16(OL.synth_bf16(seed, N, nc, col0=c0), an, np.float32(sum(w)), s=sn)
        for name, (o, ob) in one.items():
            if o is not None:
                assert _same(o[c0:c0 + nc], ef), (name, c0)
            assert np.array_equal(ob[c0:c0 + nc], eb), (name, c0)


@pytest.mark.parametrize("scored", [False, True])
def test_f32_one_launch_steps_at_the_c3_rank_layout(dev, libs, scored):
    """A C3 rank's four slots at 8 GPUs (3.2M, 3.2M, 3.2M, 0.4M) side by side,
    200 clients: every fp32 step form and the product's rounds fold with its
    waits, every column."""
    _lib, L, B = libs
    N, seed = 200, 83
    lay = overlap_layout(80_000_000, 8, "f32")
    W = lay.local_width
    st = torch.cuda.current_stream(dev).cuda_stream
    X = torch.empty((N, W), dtype=torch.float32, device=dev)
    _lib.check(B.fa_synth_f32(X.data_ptr(), N, W, W, seed, 0, 0, st), "synth", bench=True)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = None if sc is None else torch.tensor(np.array(sc, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    one = _one_launch_steps(dev, libs, X, N, W, lay, a, s, div, bf16=False)
    assert len(one) >= 9
    del X
    torch.cuda.empty_cache()
    an, sn = np.array(w, np.float32), None if sc is None else np.array(sc, np.float32)
    for c0 in range(0, W, 1 << 20):
        nc = min(1 << 20, W - c0)
        exp = OL.fedavg_f32(OL.synth_f32(seed, N, nc, col0=c0), an, np.float32(sum(w)), s=sn)
        for name, (o, _) in one.items():
            assert _same(o[c0:c0 + nc], exp), (name, c0)


@pytest.mark.parametrize("bf16", [False, True])
def test_one_launch_steps_many_small_rounds(dev, libs, bf16):
    """Eight rounds, most narrower than one pass of wide tiles (the round-tail
    forms then fold whole rounds in narrow static tiles, the segment table is
    at its largest), an odd client count, stall-aware: every step form and the
    product's rounds fold with its waits, every column."""
    from fedlesscan_amd.sharding import SlotLayout, tail_shares
    _lib, L, B = libs
    N, seed = 37, 97
    lay = SlotLayout(3_000_000, 1, 8, shares=tail_shares(8, 0.05, 5))
    W = lay.local_width
    st = torch.cuda.current_stream(dev).cuda_stream
    X = torch.empty((N, W), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
    gen = B.fa_synth_bf16 if bf16 else B.fa_synth_f32
    _lib.check(gen(X.data_ptr(), N, W, W, seed, 0, 0, st), "synth", bench=True)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = torch.tensor(np.array(sc, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    one = _one_launch_steps(dev, libs, X, N, W, lay, a, s, div, bf16=bf16)
    an, sn = np.array(w, np.float32), np.array(sc, np.float32)
    if bf16:
        ef, eb = OL.fedavg_bf16(OL.synth_bf16(seed, N, W), an, np.float32(sum(w)), s=sn)
        for name, (o, ob) in one.items():
            if o is not None:
                assert _same(o, ef), name
            assert np.array_equal(ob, eb), name
    else:
        exp = OL.fedavg_f32(OL.synth_f32(seed, N, W), an, np.float32(sum(w)), s=sn)
        for name, (o, _) in one.items():
            assert _same(o, exp), name


class _Ragged:
    """A rounds layout whose last round ends off an 8-column boundary (only
    the last round may: every round starts 8-aligned)."""

    def __init__(self, offsets):
        self.offsets = list(offsets)
        self.rounds = len(offsets) - 1

    def offset(self, k):
        return self.offsets[k]


@pytest.mark.parametrize("bf16", [False, True])
def test_one_launch_steps_ragged_last_round(dev, libs, bf16):
    """The last round's width is not a multiple of 8, so its trailing columns
    are folded by one lane with plain stores (bf16: behind that lane's release
    fence, the rest of the step being stored write-through): every step form
    and the product's rounds fold with its waits, bit for bit, and the columns
    past the last round untouched."""
    from fedlesscan_amd.sharding import ALIGN
    _lib, L, B = libs
    N, seed = 19, 41
    total = 16_384 + 8 * 8192 + 77_781          # ends 5 columns past an octet
    W = (total + ALIGN - 1) // ALIGN * ALIGN     # the row pitch (ldx)
    lay = _Ragged([0, 16_384, 16_384 + 8 * 8192, total])
    st = torch.cuda.current_stream(dev).cuda_stream
    X = torch.empty((N, W), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
    gen = B.fa_synth_bf16 if bf16 else B.fa_synth_f32
    _lib.check(gen(X.data_ptr(), N, W, W, seed, 0, 0, st), "synth", bench=True)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = torch.tensor(np.array(sc, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    one = _one_launch_steps(dev, libs, X, N, W, lay, a, s, div, bf16=bf16)
    an, sn = np.array(w, np.float32), np.array(sc, np.float32)
    if bf16:
        ef, eb = OL.fedavg_bf16(OL.synth_bf16(seed, N, W), an, np.float32(sum(w)), s=sn)
        for name, (o, ob) in one.items():
            if o is not None:
                assert _same(o[:total], ef[:total]), name
                if "copied" not in name:
                    assert np.isnan(o[total:]).all(), name
            assert np.array_equal(ob[:total], eb[:total]), name
    else:
        exp = OL.fedavg_f32(OL.synth_f32(seed, N, W), an, np.float32(sum(w)), s=sn)
        for name, (o, _) in one.items():
            assert _same(o[:total], exp[:total]), name


def test_rounds_entry_errors(dev, libs):
    """Argument errors are reported, never launched: empty or misaligned
    rounds, too many rounds, a wait before any launch or past the last
    launch's rounds, a launch under graph capture."""
    import ctypes
    _lib, L, B = libs
    st = torch.cuda.current_stream(dev).cuda_stream
    X = torch.zeros((4, 1024), dtype=torch.float32, device=dev)
    a = torch.ones(4, device=dev)
    o = torch.empty(1024, device=dev)
    r = ctypes.c_void_p()
    _lib.check(L.fa_rounds_create(ctypes.byref(r), dev.index), "create")

    def launch(offsets, rounds=None):
        offs = (ctypes.c_int64 * len(offsets))(*offsets)
        return L.fa_fedavg_f32_rounds(r, X.data_ptr(), 4, 1024, a.data_ptr(), None, 4.0, o.data_ptr(),
                                      len(offsets) - 1 if rounds is None else rounds, offs, None, st)
    with pytest.raises(ValueError):
        _lib.check(L.fa_rounds_wait(r, 0, st), "wait before launch")
    for bad in ([0, 0, 512], [0, 2, 1024], [0, 512, 1028], [0] + list(range(64, 640, 64))):
        with pytest.raises(ValueError):
            _lib.check(launch(bad), f"bad offsets {bad}")
    _lib.check(launch([0, 512, 1024]), "good")
    _lib.check(L.fa_rounds_wait(r, 1, st), "wait")
    with pytest.raises(ValueError):
        _lib.check(L.fa_rounds_wait(r, 2, st), "past the rounds")
    torch.cuda.synchronize()
    assert _same(o.cpu().numpy(), np.zeros(1024, np.float32))
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side), pytest.warns(UserWarning, match="empty"):  # the refused launch leaves it empty
        with torch.cuda.graph(g, stream=side):
            offs = (ctypes.c_int64 * 3)(0, 512, 1024)
            rc = L.fa_fedavg_f32_rounds(r, X.data_ptr(), 4, 1024, a.data_ptr(), None, 4.0, o.data_ptr(), 2, offs,
                                        None, side.cuda_stream)
    assert rc == _lib.FA_ERR_ARG
    assert L.fa_rounds_timeouts(r) == 0 and L.fa_rounds_check(r) == 0
    _lib.check(L.fa_rounds_destroy(r), "destroy")


@pytest.mark.parametrize("P", [8 * 3000 + 5, 1_000_003, 12_500_000])
def test_bf16_result_alone(dev, libs, P):
    """ABI 5: a bf16 fold stores the fp32 result, the RNE-bf16 copy or both,
    and the bf16 bits are the same either way (engine.fold_stacked(out_bf16=)
    is the per-round exchange step's call; the rounds entry: above).  Neither
    output is an argument error, not a launch."""
    from fedlesscan_amd import engine
    _lib, L, B = libs
    N, seed = 64, 71
    st = torch.cuda.current_stream(dev).cuda_stream
    ldx = (P + 63) // 64 * 64
    X = torch.empty((N, ldx), dtype=torch.bfloat16, device=dev)
    _lib.check(B.fa_synth_bf16(X.data_ptr(), N, ldx, ldx, seed, 0, 0, st), "synth", bench=True)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    both_f, both_b = engine.fold_stacked(X[:, :P], w, sc, want_bf16=True)
    alone = torch.full((P,), -1, dtype=torch.int16, device=dev).view(torch.bfloat16)
    got = engine.fold_stacked(X[:, :P], w, sc, out_bf16=alone)
    assert got is alone
    f_only = engine.fold_stacked(X[:, :P], w, sc)
    torch.cuda.synchronize()
    c = min(P, 1 << 20)
    ef, eb = OL.fedavg_bf16(OL.synth_bf16(seed, N, c), np.array(w, np.float32), np.float32(sum(w)),
                            s=np.array(sc, np.float32))
    bits = alone.view(torch.int16).cpu().numpy().view(np.uint16)
    assert np.array_equal(bits[:c], eb)
    assert np.array_equal(bits, both_b.view(torch.int16).cpu().numpy().view(np.uint16))
    assert _same(both_f.cpu().numpy()[:c], ef) and _same(f_only.cpu().numpy(), both_f.cpu().numpy())
    a = torch.tensor(np.array(w, np.float32), device=dev)
    rc = L.fa_fedavg_bf16(X.data_ptr(), N, P, ldx, a.data_ptr(), None, float(sum(w)), None, None, st)
    assert rc == _lib.FA_ERR_ARG
    import ctypes
    r = ctypes.c_void_p()
    _lib.check(L.fa_rounds_create(ctypes.byref(r), dev.index), "create")
    offs = (ctypes.c_int64 * 2)(0, P // 8 * 8)
    assert L.fa_fedavg_bf16_rounds(r, X.data_ptr(), N, ldx, a.data_ptr(), None, 1.0, None, None, 1, offs, None,
                                   st) == _lib.FA_ERR_ARG
    _lib.check(L.fa_rounds_destroy(r), "destroy")
    with pytest.raises(ValueError):
        engine.fold_rounds(X, w, sc, [0, P // 8 * 8])  # neither output
