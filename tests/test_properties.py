"""Property-based parity (hypothesis): random client counts, widths, strides,
integer and float cardinalities, stall-aware scores.

CPU part: the three oracle forms (literal reference op order, lean stacked
form, C restatement) agree bit for bit.  GPU part (-m gpu): the HIP fold
through the C-ABI agrees with them bit for bit, plus size-independent
properties of the fold that hold for ANY inputs (order of clients matters only
through the fold; a client with weight 0 changes nothing except the divisor;
duplicating every weight scales nothing)."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from fedlesscan_amd import synth
from oracle import fedavg_oracle as O
from oracle import oracle_lib as OL

weights_st = st.lists(st.one_of(st.integers(0, 5000), st.floats(0.125, 3000.0, allow_nan=False, width=32)),
                      min_size=1, max_size=40)


def _bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    na, nb = np.isnan(a), np.isnan(b)
    return a.shape == b.shape and np.array_equal(na, nb) and np.array_equal(a.view(np.uint32)[~na],
                                                                           b.view(np.uint32)[~nb])


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(w=weights_st, P=st.integers(1, 3000), seed=st.integers(0, 2**32 - 1), scored=st.booleans())
def test_oracle_forms_agree(w, P, seed, scored):
    N = len(w)
    X = synth.clients_f32(seed, N, 0, P)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    feats = [{"round_id": r} for r in synth.round_ids(seed, N, 10, 2)]
    params = [[X[i]] for i in range(N)]
    with np.errstate(all="ignore"):
        lit = (O.stall_aware_literal(feats, 10, params, w) if scored else O.fedavg_literal(params, w))[0]
        lean = O.fedavg_stacked(X, w, sc)
        c = OL.fedavg_f32(X, np.array([np.float32(x) for x in w], np.float32), np.float32(sum(w)),
                          s=None if sc is None else np.array(sc, np.float32))
    assert lit.dtype == np.float32
    assert _bits(lit, lean) and _bits(lit, c)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
torch = pytest.importorskip("torch")


@pytest.mark.gpu
@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                  HealthCheck.function_scoped_fixture])
@given(w=weights_st, P=st.integers(1, 20000), pad=st.integers(0, 70), offset=st.integers(0, 5),
       seed=st.integers(0, 2**32 - 1), scored=st.booleans())
def test_gpu_fold_matches_oracle(w, P, pad, offset, seed, scored):
    from fedlesscan_amd import engine
    dev = torch.device("cuda", 0)
    N = len(w)
    X = synth.clients_f32(seed, N, 0, P)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    big = torch.zeros((N, P + pad + offset), dtype=torch.float32, device=dev)
    big[:, offset:offset + P] = torch.from_numpy(X).to(dev)
    out = torch.full((P,), float("nan"), device=dev)
    got = engine.fold_stacked(big[:, offset:offset + P], w, sc, out=out).cpu().numpy()
    with np.errstate(all="ignore"):
        exp = O.fedavg_stacked(X, w, sc)
    assert _bits(got, exp)


@pytest.mark.gpu
@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(N=st.integers(2, 30), P=st.integers(1, 5000), seed=st.integers(0, 2**32 - 1))
def test_gpu_fold_properties(N, P, seed):
    from fedlesscan_amd import engine
    dev = torch.device("cuda", 0)
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    Xd = torch.from_numpy(X).to(dev)
    base = engine.fold_stacked(Xd, w).cpu().numpy()
    # 1. an extra client with cardinality 0 contributes x*0 = 0 to every sum: the
    #    fold value is unchanged, so the result is identical
    extra = torch.cat([Xd, Xd[:1]], 0)
    assert _bits(engine.fold_stacked(extra, w + [0]).cpu().numpy(), base)
    # 2. a single client: out = fl(fl(x*n)/fl(n)) for every column
    one = engine.fold_stacked(Xd[:1], w[:1]).cpu().numpy()
    with np.errstate(all="ignore"):
        exp = (X[0] * np.float32(w[0])) / np.float32(w[0])
    assert _bits(one, exp.astype(np.float32))
    # 3. all scores 1.0 (every result from the current round) == FedAvg
    assert _bits(engine.fold_stacked(Xd, w, [1.0] * N).cpu().numpy(), base)
    # 4. equal cardinalities and identical clients: mean of N copies of x*n over N*n
    same = Xd[:1].expand(N, P).contiguous()
    got = engine.fold_stacked(same, [7] * N).cpu().numpy()
    acc = X[0] * np.float32(7)
    s = acc.copy()
    for _ in range(N - 1):
        s = s + acc
    assert _bits(got, (s / np.float32(7 * N)).astype(np.float32))


@pytest.mark.gpu
@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(N=st.integers(60, 700), P=st.integers(1, 150_000), pad4=st.integers(0, 20), seed=st.integers(0, 2**32 - 1),
       scored=st.booleans(), cut=st.floats(0.0, 1.0))
def test_gpu_fold_many_clients(N, P, pad4, seed, scored, cut):
    """Many clients on 16-B aligned rows: the LDS-staged folds' multi-chunk,
    two-chunks-in-flight paths and their partial last chunk, as one fold and
    as a two-part chunked continuation (fa_fold_f32), against the C oracle."""
    from fedlesscan_amd import _lib
    L = _lib.load()
    dev = torch.device("cuda", 0)
    ldx = P + (-P) % 4 + 4 * pad4
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    big = torch.zeros((N, ldx), dtype=torch.float32, device=dev)
    big[:, :P] = torch.from_numpy(X).to(dev)
    a = torch.tensor([float(np.float32(x)) for x in w], dtype=torch.float32, device=dev)
    s = None if sc is None else torch.tensor([float(np.float32(x)) for x in sc], dtype=torch.float32, device=dev)
    div = float(np.float32(sum(w)))
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = torch.full((P,), float("nan"), device=dev)
    _lib.check(L.fa_fedavg_f32(big.data_ptr(), N, P, ldx, a.data_ptr(), None if s is None else s.data_ptr(), div,
                               out.data_ptr(), stream), "fold")
    assert _bits(out.cpu().numpy(), exp)
    k = max(1, min(N - 1, int(cut * N)))  # rows [0, k) then [k, N), accumulator carried
    acc = torch.full((P,), float("nan"), device=dev)
    _lib.check(L.fa_fold_f32(big.data_ptr(), k, P, ldx, a.data_ptr(), None if s is None else s.data_ptr(), None,
                             div, 0, acc.data_ptr(), stream), "part 1")
    _lib.check(L.fa_fold_f32(big[k].data_ptr(), N - k, P, ldx, a[k:].data_ptr(),
                             None if s is None else s[k:].data_ptr(), acc.data_ptr(), div, 1, acc.data_ptr(),
                             stream), "part 2")
    assert _bits(acc.cpu().numpy(), exp)


@pytest.mark.gpu
@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                  HealthCheck.function_scoped_fixture])
@given(w=weights_st, P=st.integers(1, 50000), seed=st.integers(0, 2**32 - 1), scored=st.booleans(),
       chunk_rows=st.integers(1, 12), slots=st.integers(2, 6), announce=st.sampled_from(["none", "exact", "off"]),
       cuts=st.lists(st.floats(0, 1), max_size=4))
def test_gpu_native_ingest_matches_oracle(w, P, seed, scored, chunk_rows, slots, announce, cuts):
    """The native ingest pipe over random rows split into random pieces, random
    chunk sizes, slot counts and announced row counts: bit-exact against the C
    oracle with numpy's weight rounding."""
    from fedlesscan_amd.ingest import NativeStreamingFold
    dev = torch.device("cuda", 0)
    N = len(w)
    X = synth.clients_f32(seed, N, 0, P)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    ldx = (P + 63) // 64 * 64
    exp_rows = {"none": 0, "exact": N, "off": N + 3}[announce]
    sf = NativeStreamingFold(P, dev, chunk_bytes=chunk_rows * ldx * 4, slots=slots, expected_rows=exp_rows)
    edges = sorted({0, P, *(int(c * P) for c in cuts)})
    for i in range(N):
        sf.add([X[i, a:b] for a, b in zip(edges, edges[1:])], w[i], None if sc is None else sc[i])
    with np.errstate(all="ignore"):
        got = sf.finish().cpu().numpy()
        exp = OL.fedavg_f32(X, np.array([np.float32(x) for x in w], np.float32), np.float32(sum(w)),
                            s=None if sc is None else np.array(sc, np.float32))
    assert _bits(got, exp)
