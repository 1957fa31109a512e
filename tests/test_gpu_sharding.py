"""The multi-GPU path with the HIP fold on the MI355X.

The 8-GPU run belongs to the driver; here the same code runs on the one GPU
of the box:
  - world size 1: ShardedAggregator with its default fold (engine.fold_stacked
    -> libfedavg_hip.so) over round-robin slots, fp32 and bf16 (the bf16 model
    is exchanged as RNE bf16), and the reference-shaped per-layer entry;
  - world size 2, both ranks on cuda:0, gloo exchange (host-staged): every
    rank folds its own slots with the HIP kernels and reassembles the model.
Everything bit-exact against the oracle.
"""
import os
import socket

import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _scores(seed, n):
    return [(r + 1) / 11 for r in synth.round_ids(seed, n, 10, 2)]


@pytest.mark.parametrize("one_launch", [True, False, "auto"])
@pytest.mark.parametrize("P,rounds,scored", [(10007, 3, False), (4096, 4, True), (1, 1, False), (300001, 8, True)])
def test_slots_world1_fp32(P, rounds, scored, one_launch):
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    from oracle import oracle_lib as OL
    dev = torch.device("cuda", 0)
    N, seed = 37, 5
    lay = SlotLayout(P, 1, rounds)
    X = torch.zeros((N, lay.local_width), dtype=torch.float32, device=dev)
    Xh = synth.clients_f32(seed, N, 0, P)
    for k, (lo, hi) in enumerate(lay.slots(0)):
        if hi > lo:
            X[:, k * lay.sub:k * lay.sub + hi - lo] = torch.from_numpy(Xh[:, lo:hi]).to(dev)
    w = synth.cardinalities(seed, N)
    sc = _scores(seed, N) if scored else None
    full = ShardedAggregator(one_launch=one_launch).aggregate_slots(X, w, sc, lay)
    exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert G.same_bits(full.cpu().numpy(), exp)


@pytest.mark.parametrize("one_launch", [True, False, "auto"])
@pytest.mark.parametrize("P,rounds", [(8 * 1000 + 3, 2), (65536, 4), (1_000_003, 5)])
def test_slots_world1_bf16_exchange(P, rounds, one_launch):
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    from oracle import fedavg_oracle as O
    dev = torch.device("cuda", 0)
    N, seed = 29, 6
    lay = SlotLayout(P, 1, rounds)
    X = torch.zeros((N, lay.local_width), dtype=torch.int16, device=dev)
    Xb = synth.clients_bf16(seed, N, 0, P)
    for k, (lo, hi) in enumerate(lay.slots(0)):
        if hi > lo:
            X[:, k * lay.sub:k * lay.sub + hi - lo] = torch.from_numpy(Xb[:, lo:hi].view(np.int16)).to(dev)
    w = synth.cardinalities(seed, N)
    sc = _scores(seed, N)
    full = ShardedAggregator(one_launch=one_launch).aggregate_slots(X.view(torch.bfloat16), w, sc, lay)
    assert full.dtype == torch.bfloat16
    _, expb = O.fedavg_stacked_bf16(Xb, w, sc)
    assert np.array_equal(full.view(torch.int16).cpu().numpy().view(np.uint16), expb)


def _slots_input(bf16, N, P, seed, lay, dev):
    """X [N, lay.local_width] on the GPU holding rank 0's slots, and the
    oracle's expected bits (fp32 as uint32, bf16 as the RNE uint16 model)."""
    from oracle import fedavg_oracle as O
    w = synth.cardinalities(seed, N)
    sc = _scores(seed, N)
    if bf16:
        X = torch.zeros((N, lay.local_width), dtype=torch.int16, device=dev)
        Xb = synth.clients_bf16(seed, N, 0, P)
        src = Xb.view(np.int16)
        _, exp = O.fedavg_stacked_bf16(Xb, w, sc)
    else:
        X = torch.zeros((N, lay.local_width), dtype=torch.float32, device=dev)
        src = synth.clients_f32(seed, N, 0, P)
        exp = O.fedavg_stacked(src, w, sc).view(np.uint32)
    for k, (lo, hi) in enumerate(lay.slots(0)):
        if hi > lo:
            X[:, lay.offset(k):lay.offset(k) + hi - lo] = torch.from_numpy(src[:, lo:hi]).to(dev)
    return (X.view(torch.bfloat16) if bf16 else X), w, sc, exp


def _bits(full, bf16):
    return full.view(torch.int16).cpu().numpy().view(np.uint16) if bf16 else full.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("bf16", [False, True])
def test_probe_step_form_settles_records_and_stays_exact(bf16, monkeypatch):
    """one_launch="probe": the first PROBE_STEPS calls of a shape alternate
    the one launch and per-round launches (PROBE_WARM untimed calls of each,
    then PROBE_CALLS timed ones), later calls keep the
    faster, and the choice is recorded: a fresh "auto" aggregator (a later
    process's) runs it without probing.  Every call bit-exact; a new shape
    probes anew."""
    from fedlesscan_amd import engine
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    dev = torch.device("cuda", 0)
    agg = ShardedAggregator(one_launch="probe")
    assert ShardedAggregator().one_launch == "auto"
    # shapes no other test uses: the cache file is shared by the session (conftest),
    # and a record another test left for the same key would settle the probe early
    for P, rounds in ((300_001, 4), (65_544, 3)):
        N, seed = 33, 9
        lay = SlotLayout(P, 1, rounds)
        Xin, w, sc, exp = _slots_input(bf16, N, P, seed, lay, dev)
        for call in range(ShardedAggregator.PROBE_STEPS + 2):
            settled = agg.step_form(Xin, lay)
            assert (settled is None) == (call < ShardedAggregator.PROBE_STEPS), (call, settled)
            assert np.array_equal(_bits(agg.aggregate_slots(Xin, w, sc, lay), bf16), exp), (P, call)
        form = agg.step_form(Xin, lay)
        assert form in ("one launch", "per round")
        # a fresh aggregator finds the record and times nothing
        fresh = ShardedAggregator()
        assert fresh.step_form(Xin, lay) == form
        calls = []
        real = engine.fold_rounds
        monkeypatch.setattr(engine, "fold_rounds", lambda *a, **k: calls.append(1) or real(*a, **k))
        monkeypatch.setattr(torch.cuda.Event, "elapsed_time", lambda *a: pytest.fail("a probe timed a call"))
        assert np.array_equal(_bits(fresh.aggregate_slots(Xin, w, sc, lay), bf16), exp)
        assert len(calls) == (1 if form == "one launch" else 0)
        monkeypatch.undo()
    with pytest.raises(ValueError):
        ShardedAggregator(one_launch="sometimes")


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("recorded", ["one", "per", None])
def test_step_form_restored_from_the_cache_file(bf16, recorded, monkeypatch):
    """A "fedavg-step" line another process wrote to the tuner's cache file:
    a fresh process (the cache re-read) with one_launch="auto" runs that form
    from its first call -- no probe, no timing -- and is bit-exact; with no
    line it runs per-round launches."""
    from fedlesscan_amd import _lib, engine
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    dev = torch.device("cuda", 0)
    # a key of its own per case (P): this process already holds what earlier cases recorded
    N, seed = 70, 31 + (recorded == "one")
    P = 200_003 + (8 if bf16 else 0) + {"one": 0, "per": 4096, None: 8192}[recorded]
    lay = SlotLayout(P, 1, 4)
    Xin, w, sc, exp = _slots_input(bf16, N, P, seed, lay, dev)
    agg = ShardedAggregator()
    key = agg.step_key(Xin, lay)
    path = os.environ["FEDAVG_TUNE_CACHE"]
    if recorded:
        with open(path, "a") as f:
            f.write(f"fedavg-step 1 {_lib.ABI_VERSION} {key} {recorded}\n")
    _lib.call("fa_tune_cache_path", path.encode())  # as a new process: the file is read on the next lookup
    calls = []
    real = engine.fold_rounds
    monkeypatch.setattr(engine, "fold_rounds", lambda *a, **k: calls.append(1) or real(*a, **k))
    monkeypatch.setattr(torch.cuda.Event, "elapsed_time", lambda *a: pytest.fail("a probe timed a call"))
    assert np.array_equal(_bits(agg.aggregate_slots(Xin, w, sc, lay), bf16), exp)
    assert len(calls) == (1 if recorded == "one" else 0)
    assert agg.step_form(Xin, lay) == {"one": "one launch", "per": "per round", None: None}[recorded]


def _c4_rank_input(dev, N=256, seed=52):
    """A C4 rank's share as 4 rounds (~1 ms of fold) at world 1, in HBM."""
    from fedlesscan_amd.sharding import overlap_layout
    B = __import__("fedlesscan_amd._lib", fromlist=["x"]).load_bench()
    lay = overlap_layout(100_000_000 // 8, 1, "bf16")
    W = lay.local_width
    X = torch.empty((N, W), dtype=torch.bfloat16, device=dev)
    assert B.fa_synth_bf16(X.data_ptr(), N, W, W, seed, 0, 0, torch.cuda.current_stream(dev).cuda_stream) == 0
    return lay, X, synth.cardinalities(seed, N), _scores(seed, N)


def _hold_the_fold(busy):
    """~5 ms of work ahead of the step on the caller's stream: the fold (and the
    waiters' clocks, which start with it) begins only after the host has
    enqueued the whole step, so every wait sees an unfinished round however
    slowly this process issues its first calls."""
    for _ in range(24):
        busy.fill_(1.0)


def test_round_wait_timeout_raises_on_every_path(monkeypatch):
    """A round wait that gives up (a tick limit far below one C4-slot fold,
    FEDAVG_ROUND_WAIT_US) lets the exchange behind it read an unfinished
    round: aggregate_slots raises AggregationError instead of returning the
    model (check="sync"), or check_timeouts() does (check="deferred").  At
    world 1 the waits are the peer exchange's (the RCCL step folds its slots
    straight into the model and has nothing to wait for there; its waits at
    world 2: test_round_wait_timeout_two_ranks).  At the default limit the
    same steps are bit-exact against the oracle, every column."""
    from fedlesscan_amd.aggregator.exceptions import AggregationError
    from fedlesscan_amd.sharding import ShardedAggregator
    from oracle import oracle_lib as OL
    dev = torch.device("cuda", 0)
    N, seed = 256, 52
    lay, X, w, sc = _c4_rank_input(dev, N, seed)
    monkeypatch.setenv("FEDAVG_ROUND_WAIT_US", "1")  # read when the peer exchange's state is created
    busy = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    sync = ShardedAggregator(one_launch=True, exchange="peer_copy")
    deferred = ShardedAggregator(one_launch=True, exchange="peer_copy", check="deferred")
    for agg in (sync, deferred):
        # a first call creates the peer exchange (which synchronises the device):
        # timed out or not, it is not the call under test
        try:
            agg.aggregate_slots(X, w, sc, lay)
            agg.check_timeouts()
        except AggregationError:
            pass
    _hold_the_fold(busy)
    with pytest.raises(AggregationError, match="timed out"):
        sync.aggregate_slots(X, w, sc, lay)
    _hold_the_fold(busy)
    out = deferred.aggregate_slots(X, w, sc, lay)
    assert out.dtype == torch.bfloat16
    with pytest.raises(AggregationError, match="timed out"):
        deferred.check_timeouts()
    deferred.check_timeouts()  # nothing left unchecked
    torch.cuda.synchronize()
    sync.close()
    deferred.close()
    del busy, out
    monkeypatch.delenv("FEDAVG_ROUND_WAIT_US")
    peer = ShardedAggregator(one_launch=True, exchange="peer_copy")
    got_peer = _bits(peer.aggregate_slots(X, w, sc, lay), True)
    got_one = _bits(ShardedAggregator(one_launch=True).aggregate_slots(X, w, sc, lay), True)
    peer.close()
    del X
    torch.cuda.empty_cache()
    an, sn = np.array(w, np.float32), np.array(sc, np.float32)
    P = lay.P  # world 1: global column p is local column p
    expb = np.empty(P, np.uint16)
    for c0 in range(0, P, 1 << 21):
        nc = min(1 << 21, P - c0)
        _, expb[c0:c0 + nc] = OL.fedavg_bf16(OL.synth_bf16(seed, N, nc, col0=c0), an, np.float32(sum(w)), s=sn)
    assert np.array_equal(got_peer, expb) and np.array_equal(got_one, expb)


def _timeout_rank(rank, world, port, q):
    """One of two ranks sharing the GPU: the RCCL-form one-launch step with a
    1 us round-wait limit must raise on BOTH ranks (the MAX over the group)."""
    import torch as T
    import torch.distributed as dist
    from fedlesscan_amd.aggregator.exceptions import AggregationError
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FEDAVG_ROUND_WAIT_US="1")
    T.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = T.device("cuda", 0)
        N, P = 256, 4_000_000
        lay = SlotLayout(P, world, 4)
        B = __import__("fedlesscan_amd._lib", fromlist=["x"]).load_bench()
        W = lay.local_width
        X = T.empty((N, W), dtype=T.bfloat16, device=dev)
        assert B.fa_synth_bf16(X.data_ptr(), N, W, W, 5, 0, 0, T.cuda.current_stream(dev).cuda_stream) == 0
        w = synth.cardinalities(5, N)
        busy = T.empty(1 << 28, dtype=T.float32, device=dev)
        res = []
        for check in ("sync", "deferred"):
            agg = ShardedAggregator(one_launch=True, check=check)
            try:  # a first call creates the rounds state (a device synchronisation): not the call under test
                agg.aggregate_slots(X, w, None, lay)
                agg.check_timeouts()
            except AggregationError:
                pass
            _hold_the_fold(busy)
            try:
                agg.aggregate_slots(X, w, None, lay)
                if check == "deferred":
                    agg.check_timeouts()
                res.append("returned")
            except AggregationError as e:
                res.append("raised" if "timed out" in str(e) else repr(e))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_round_wait_timeout_two_ranks():
    """The RCCL exchange's round waits at world 2 (two gloo ranks sharing the
    GPU): with a 1 us limit every rank raises, in both check modes."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: ["raised", "raised"], 1: ["raised", "raised"]}, got


@pytest.mark.parametrize("one_launch", ["auto", True])
@pytest.mark.parametrize("bf16", [False, True])
def test_aggregate_slots_captures_into_hip_graph(one_launch, bf16):
    """Under a HIP graph capture aggregate_slots takes the per-round launches
    (the one launch refuses capture: its epochs would replay) and times
    nothing; the graph replays bit-exactly on new client rows."""
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    dev = torch.device("cuda", 0)
    N, P = 24, 100_003
    lay = SlotLayout(P, 1, 4)
    Xin, w, sc, _ = _slots_input(bf16, N, P, 61, lay, dev)
    agg = ShardedAggregator(one_launch=one_launch)
    agg.aggregate_slots(Xin, w, sc, lay)  # the tuner's first calls of the slot shapes, outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        full = agg.aggregate_slots(Xin, w, sc, lay)
    for seed in (62, 63):
        src, _, _, exp = _slots_input(bf16, N, P, seed, lay, dev)
        Xin.copy_(src)
        g.replay()
        torch.cuda.synchronize()
        got = _bits(full, bf16)
        # the weights are the captured ones (seed 61's); the expected bits with them
        from oracle import fedavg_oracle as O
        if bf16:
            _, exp = O.fedavg_stacked_bf16(synth.clients_bf16(seed, N, 0, P), w, sc)
        else:
            exp = O.fedavg_stacked(synth.clients_f32(seed, N, 0, P), w, sc).view(np.uint32)
        assert np.array_equal(got, exp), seed


@pytest.mark.parametrize("what", ["step", "fold"])
@pytest.mark.parametrize("bf16", [False, True])
def test_captured_graph_replays_stay_exact(what, bf16):
    """A captured step (aggregate_slots: per-round launches) or a captured
    fold_stacked, replayed 40 times over fresh client rows, equals the eager
    call on the same rows every time (the captured factors live in memory the
    graph owns)."""
    from fedlesscan_amd import engine
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    dev = torch.device("cuda", 0)
    N, P = 24, 100_003
    lay = SlotLayout(P, 1, 4)
    Xin, w, sc, _ = _slots_input(bf16, N, P, 61, lay, dev)
    if what == "fold":
        Xin = Xin[:, :25_001]
    agg, eager = ShardedAggregator(one_launch=True), ShardedAggregator(one_launch=False)

    def run(a):
        if what == "step":
            return a.aggregate_slots(Xin, w, sc, lay)
        return engine.fold_stacked(Xin, w, sc, out_bf16=torch.empty(Xin.shape[1], dtype=torch.bfloat16, device=dev)) \
            if bf16 else engine.fold_stacked(Xin, w, sc)

    run(agg)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        full = run(agg)
    iv = torch.int16 if bf16 else torch.int32
    gen = torch.Generator(device=dev)
    bad = []
    for i in range(40):
        gen.manual_seed(100 + i)
        Xin.copy_(torch.randn(Xin.shape, generator=gen, device=dev, dtype=torch.float32).to(Xin.dtype))
        g.replay()
        exp = run(eager)
        torch.cuda.synchronize()
        diff = (full.view(iv) != exp.view(iv)).nonzero()
        if diff.numel():
            bad.append((i, int(diff.numel()), int(diff[0]), int(diff[-1]), int((full.view(iv)[diff] == 0).sum())))
    assert not bad, bad


@pytest.mark.parametrize("one_launch", [True, False])
@pytest.mark.parametrize("bf16", [False, True])
def test_quantised_layout_world1(one_launch, bf16):
    """Rounds in whole quanta (SlotLayout quantum), both step forms, bit-exact."""
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout, tail_shares
    from oracle import fedavg_oracle as O
    dev = torch.device("cuda", 0)
    N, P, seed = 45, 300_001, 14
    lay = SlotLayout(P, 1, 4, shares=tail_shares(4, 0.25), quantum=4096)
    assert all(w % 4096 == 0 for w in lay.widths[:-1])
    w = synth.cardinalities(seed, N)
    sc = _scores(seed, N)
    if bf16:
        X = torch.zeros((N, lay.local_width), dtype=torch.int16, device=dev)
        Xb = synth.clients_bf16(seed, N, 0, P)
        src = Xb.view(np.int16)
        _, exp = O.fedavg_stacked_bf16(Xb, w, sc)
    else:
        X = torch.zeros((N, lay.local_width), dtype=torch.float32, device=dev)
        src = synth.clients_f32(seed, N, 0, P)
        exp = O.fedavg_stacked(src, w, sc).view(np.uint32)
    for k, (lo, hi) in enumerate(lay.slots(0)):
        if hi > lo:
            X[:, lay.offset(k):lay.offset(k) + hi - lo] = torch.from_numpy(src[:, lo:hi]).to(dev)
    full = ShardedAggregator(one_launch=one_launch).aggregate_slots(X.view(torch.bfloat16) if bf16 else X, w, sc, lay)
    got = full.view(torch.int16).cpu().numpy().view(np.uint16) if bf16 else full.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, exp)


def test_aggregate_layers_world1_matches_reference_goldens():
    """The reference's own fixture shapes through the sharded per-layer entry."""
    from fedlesscan_amd.sharding import ShardedAggregator
    case = "f32_small"
    m = G.manifest()[case]
    out = ShardedAggregator().aggregate_layers(G.parameters(case), m["weights"])
    exp = G.expected(case, "fedavg")
    assert len(out) == len(exp)
    assert all(a.shape == b.shape and G.same_bits(a, b) for a, b in zip(out, exp))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _misaligned(X):
    """The same values in a view that is NOT 16-B aligned and whose row pitch
    is off the quad / octet grid (one element of padding per row, one of
    offset): the one launch cannot read it as it is."""
    N, W = X.shape
    base = torch.empty(N * (W + 1) + 1, dtype=X.dtype, device=X.device)
    V = base[1:].view(N, W + 1)[:, :W]
    V.copy_(X)
    assert V.data_ptr() % 16 != 0 and V.stride(0) % 4 != 0
    return V


def _rank(rank, world, port, N, P, rounds, seed, bf16, q, exchange="rccl", misalign=False):
    import torch as T
    import torch.distributed as dist
    from fedlesscan_amd.sharding import ShardedAggregator, SlotLayout
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    T.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = T.device("cuda", 0)
        lay = SlotLayout(P, world, rounds)
        if bf16:
            X = T.zeros((N, lay.local_width), dtype=T.int16, device=dev)
        else:
            X = T.zeros((N, lay.local_width), dtype=T.float32, device=dev)
        for k, (lo, hi) in enumerate(lay.slots(rank)):
            if hi > lo:
                part = (synth.clients_bf16(seed, N, lo, hi - lo).view(np.int16) if bf16
                        else synth.clients_f32(seed, N, lo, hi - lo))
                X[:, k * lay.sub:k * lay.sub + hi - lo] = T.from_numpy(part).to(dev)
        w = synth.cardinalities(seed, N)
        sc = _scores(seed, N)
        Xin = X.view(T.bfloat16) if bf16 else X
        outs = []
        if misalign:
            # rank 1 hands over rows the one launch cannot
            # read as they are; the group still takes one form (rank 1 folds
            # an aligned copy), so every rank issues the same collectives --
            # the sync check's all-reduce included -- and nobody hangs
            if rank == 1:
                Xin = _misaligned(Xin)
            agg = ShardedAggregator(one_launch=True, exchange=exchange)
            fulls = [agg.aggregate_slots(Xin, w, sc, lay) for _ in range(3)]
            outs = [f.view(T.int16 if bf16 else T.int32).cpu().numpy().tobytes() for f in fulls]
            agg.close()
        elif exchange == "rccl":
            agg = ShardedAggregator(one_launch="probe")  # the probe's all-reduce runs over the group
            for _ in range(ShardedAggregator.PROBE_STEPS + 1):
                full = agg.aggregate_slots(Xin, w, sc, lay)
                outs.append(full.view(T.int16 if bf16 else T.int32).cpu().numpy().tobytes())
            assert agg.step_form(Xin, lay) in ("one launch", "per round")
        else:
            # the peer-copy exchange: IPC-opened send buffers, flags polled across
            # processes, copy-engine pulls; steps back to back (the fence keeps a
            # send buffer until every peer has pulled it), then sync and deferred
            agg = ShardedAggregator(one_launch=True, exchange=exchange)
            fulls = [agg.aggregate_slots(Xin, w, sc, lay) for _ in range(4)]
            outs = [f.view(T.int16 if bf16 else T.int32).cpu().numpy().tobytes() for f in fulls]
            deferred = ShardedAggregator(one_launch=True, exchange=exchange, check="deferred")
            fulls = [deferred.aggregate_slots(Xin, w, sc, lay) for _ in range(3)]
            deferred.check_timeouts()
            outs += [f.view(T.int16 if bf16 else T.int32).cpu().numpy().tobytes() for f in fulls]
            assert len(agg._peers) == 1 and next(iter(agg._peers.values())) is not None
            agg.close()
            deferred.close()
        assert all(o == outs[0] for o in outs)
        q.put((rank, outs[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("misalign", [False, True])
@pytest.mark.parametrize("exchange", ["rccl", "peer_copy"])
@pytest.mark.parametrize("bf16", [False, True])
def test_two_ranks_on_one_gpu(bf16, exchange, misalign):
    """Two ranks share the GPU over gloo: the slot exchange through the group
    ("rccl": gloo host-staged here), or the kernel-free peer copy (IPC handles
    of the same device, cross-process flags and acks), bit-exact; misalign:
    rank 1's rows are a 16-B-misaligned view."""
    import torch.multiprocessing as mp
    from oracle import fedavg_oracle as O
    N, P, rounds, seed, world = 17, 20011, 3, 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, N, P, rounds, seed, bf16, q, exchange, misalign))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = synth.cardinalities(seed, N)
    sc = _scores(seed, N)
    if bf16:
        _, exp = O.fedavg_stacked_bf16(synth.clients_bf16(seed, N, 0, P), w, sc)
        for r in range(world):
            assert np.array_equal(np.frombuffer(got[r], dtype=np.uint16), exp), r
    else:
        exp = O.fedavg_stacked(synth.clients_f32(seed, N, 0, P), w, sc)
        for r in range(world):
            assert np.array_equal(np.frombuffer(got[r], dtype=np.uint32), exp.view(np.uint32)), r
