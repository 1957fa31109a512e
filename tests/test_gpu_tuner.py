"""The measured form choice (fa_set_autotune, csrc/fold_kernels.hpp Tuner).

The first calls of a new shape each run one candidate kernel form between two
events; once every candidate has its samples the shape runs the fastest.  All
forms compute the same bits, so every call of a shape -- whichever candidate
it ran -- must be bit-identical to the oracle (the fold of
fed_avg_aggregator.py:24-42 / stall_aware_aggregation.py:42-67).  The shapes
below are called until their measurement is complete, so every candidate form
runs on each of them: narrow (LDS forms), a few tiles per CU (every form),
large (grid-stride forms), P % 4 / P % 8 tails, a padded row pitch, one client.
"""
import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth
from oracle import oracle_lib as OL  # checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

F32_SHAPES = [  # (N, P, ldx pad, scored)
    (1, 1003, 0, False),
    (3, 4099, 0, True),
    (17, 70001, 0, False),
    (33, 65536 * 4 + 5, 0, True),
    (64, 909123, 0, False),
    (300, 1048579, 0, True),
    (1024, 65536, 0, False),
    (10, 5000, 120, False),
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


def _run_until_tuned(L, fold, form, max_calls=80):
    """Call fold() until fa_fold_form names a form; returns the outputs of every call."""
    outs = []
    for _ in range(max_calls):
        outs.append(fold())
        torch.cuda.synchronize()
        if form():
            break
    return outs


@pytest.mark.parametrize("N,P,pad,scored", F32_SHAPES)
def test_f32_every_candidate_bit_exact(dev, L, N, P, pad, scored):
    seed = 71 + N
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    ldx = P + pad
    Xd = torch.zeros((N, ldx), dtype=torch.float32, device=dev)
    Xd[:, :P] = torch.from_numpy(X).to(dev)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = None if sc is None else torch.tensor(np.array(sc, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    from fedlesscan_amd import _lib

    def fold():
        o = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
        _lib.check(L.fa_fedavg_f32(Xd.data_ptr(), N, P, ldx, a.data_ptr(), None if s is None else s.data_ptr(),
                                   div, o.data_ptr(), st), "fa_fedavg_f32")
        return o

    form = lambda: L.fa_fold_form(1, N, P, ldx, 1 if scored else 0, st).decode()  # noqa: E731
    outs = _run_until_tuned(L, fold, form)
    assert form(), f"{N} x {P}: measurement did not complete in {len(outs)} calls"
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    for k, o in enumerate(outs):
        assert G.same_bits(o.cpu().numpy(), exp), (N, P, k)
    # the measured shape keeps its form: a later call is bit-exact too
    assert G.same_bits(fold().cpu().numpy(), exp)


@pytest.mark.parametrize("N,P,scored", BF16_SHAPES)
def test_bf16_every_candidate_bit_exact(dev, L, N, P, scored):
    seed = 91 + N
    Xb = synth.clients_bf16(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    ldx = (P + 7) // 8 * 8
    Xd = torch.zeros((N, ldx), dtype=torch.int16, device=dev)
    Xd[:, :P] = torch.from_numpy(Xb.view(np.int16)).to(dev)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    s = None if sc is None else torch.tensor(np.array(sc, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    from fedlesscan_amd import _lib

    def fold():
        o = torch.full((P,), float("nan"), dtype=torch.float32, device=dev)
        ob = torch.zeros((P,), dtype=torch.int16, device=dev)
        _lib.check(L.fa_fedavg_bf16(Xd.data_ptr(), N, P, ldx, a.data_ptr(), None if s is None else s.data_ptr(),
                                    div, o.data_ptr(), ob.data_ptr(), st), "fa_fedavg_bf16")
        return o, ob

    form = lambda: L.fa_fold_form(2, N, P, ldx, 1 if scored else 0, st).decode()  # noqa: E731
    outs = _run_until_tuned(L, fold, form)
    assert form(), f"bf16 {N} x {P}: measurement did not complete in {len(outs)} calls"
    ef, eb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)),
                            s=None if sc is None else np.array(sc, np.float32))
    for k, (o, ob) in enumerate(outs):
        assert G.same_bits(o.cpu().numpy(), ef), (N, P, k)
        assert np.array_equal(ob.cpu().numpy().view(np.uint16), eb), (N, P, k)


def test_hostf_and_engine_path_tuned(dev, L):
    """engine.fold_stacked (the drop-in's path, *_hostf entries) goes through the
    tuner too: repeated calls of one shape stay bit-exact while it measures."""
    from fedlesscan_amd import engine
    N, P = 48, 600_007
    X = synth.clients_f32(5, N, 0, P)
    w = synth.cardinalities(5, N)
    Xd = torch.from_numpy(X).to(dev)
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)))
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(60):
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
