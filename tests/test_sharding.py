"""Multi-rank path on CPU (gloo, world_size 2 and 3): bucket partition, local
fold of each bucket, all-gather reassembly.  The per-rank fold is the oracle
here (no GPU in this container); the GPU fold itself is covered by
test_gpu_parity.py.  Bit-exact against the oracle over the full matrix."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fedlesscan_amd import synth
from fedlesscan_amd.sharding import (ShardedAggregator, SlotLayout, bucket_bounds, chunk_size, overlap_layout,
                                     tail_shares)


def test_bucket_bounds_cover_and_align():
    for P in (0, 1, 63, 64, 65, 1000, 10_000_000, 12_345_679):
        for world in (1, 2, 3, 4, 7, 8):
            b = bucket_bounds(P, world)
            assert len(b) == world
            assert b[0][0] == 0 and b[-1][1] == P
            for (l0, h0), (l1, h1) in zip(b, b[1:]):
                assert h0 == l1 and l0 <= h0
            c = chunk_size(P, world)
            nonempty = [hi - lo for lo, hi in b if hi > lo]
            assert all(x == c for x in nonempty[:-1])
            assert all(lo % 64 == 0 for lo, hi in b if hi > lo)


def test_slot_layout_partitions_the_vector():
    for P in (1, 64, 1000, 10007, 10_000_000):
        for world in (1, 2, 3, 8):
            for rounds, tail in ((1, 1), (2, 1), (4, 1), (2, 0.5), (4, 0.25), (4, 0.01), (8, 0.125)):
                lay = SlotLayout(P, world, rounds, shares=tail_shares(rounds, tail))
                assert lay.local_width == sum(lay.widths) and lay.padded_total == world * lay.local_width
                assert all(w % 64 == 0 for w in lay.widths)
                assert [lay.offset(k) for k in range(rounds)] == [sum(lay.widths[:k]) for k in range(rounds)]
                if tail == 1:
                    assert lay.uniform and lay.widths == [lay.sub] * rounds
                elif P >= 64 * world * rounds * 100:  # big enough for the ratio to show through the alignment
                    assert lay.widths[-1] < lay.widths[0]
                    assert abs(lay.widths[-1] / lay.widths[0] - tail) < 0.02
                # no round is wholly padding beyond what one aligned unit per slot needs
                assert world * (lay.local_width - len(lay.widths) * 64) < P + 64 * world * rounds
                cover = []
                for r in range(world):
                    for k, (lo, hi) in enumerate(lay.slots(r)):
                        if hi == lo:
                            continue  # slot entirely past P
                        assert lo % 64 == 0
                        rlo, rhi = lay.round_range(k)
                        assert rlo <= lo <= hi <= rhi
                        cover.append((lo, hi))
                cover.sort()
                pos = 0
                for lo, hi in cover:
                    if hi > lo:
                        assert lo == pos
                        pos = hi
                assert pos == P
                if rounds == 1:
                    assert [lay.slot(r, 0) for r in range(world)] == bucket_bounds(P, world)


def test_quantized_slot_layout():
    """quantum: every round but the last a whole number of quanta (the nearest,
    at least one), the last the rest; the rounds still partition [0, P)."""
    from fedlesscan_amd.sharding import pass_quantum
    assert pass_quantum(256, "bf16") == 2_097_152 and pass_quantum(256, "f32") == 1_048_576
    lay = overlap_layout(100_000_000, 8, "bf16", quantum=pass_quantum(256, "bf16"))
    assert lay.widths == [4_194_304, 4_194_304, 2_097_152, 2_014_400]
    assert lay.local_width == overlap_layout(100_000_000, 8, "bf16").local_width
    lay = overlap_layout(80_000_000, 8, quantum=pass_quantum(256, "f32"))
    assert lay.widths == [3_145_728] * 3 + [562_816]
    for P, world, rounds, q in ((10007, 2, 4, 128), (1_000_003, 3, 4, 4096), (64 * 8 * 5, 8, 4, 64),
                                (300_000, 2, 3, 65536)):
        lay = SlotLayout(P, world, rounds, shares=tail_shares(rounds, 0.25), quantum=q)
        assert all(w % q == 0 and w >= q for w in lay.widths[:-1]) and lay.widths[-1] >= 64
        assert world * lay.local_width >= P
        cover = sorted((lo, hi) for r in range(world) for lo, hi in lay.slots(r) if hi > lo)
        pos = 0
        for lo, hi in cover:
            assert lo == pos
            pos = hi
        assert pos == P
    with pytest.raises(ValueError):
        SlotLayout(10007, 2, 4, quantum=100)  # not a multiple of the alignment
    with pytest.raises(ValueError):
        SlotLayout(1000, 2, 4, quantum=64 * 64)  # four rounds of quanta do not fit


def test_tail_shares():
    assert tail_shares(4, 1.0) == [1.0] * 4
    assert tail_shares(4, 0.25) == [1.0, 1.0, 1.0, 0.25]
    assert tail_shares(4, 0.25, 2) == [1.0, 1.0, 0.5, 0.25]
    assert tail_shares(1, 0.25, 2) == [1.0]
    sh = tail_shares(4, 0.125, 9)  # steps capped at rounds - 1
    assert sh[0] == 1.0 and abs(sh[-1] - 0.125) < 1e-12 and sh == sorted(sh, reverse=True)
    with pytest.raises(ValueError):
        tail_shares(4, 0.0)
    lay = SlotLayout(100_000_000, 8, 4, shares=tail_shares(4, 0.25, 2))
    w = lay.widths
    assert w[0] == w[1] and abs(w[2] / w[0] - 0.5) < 1e-3 and abs(w[3] / w[0] - 0.25) < 1e-3
    assert lay.round_range(3)[1] == lay.padded_total >= 100_000_000
    assert overlap_layout(100_000_000, 8, "bf16").widths == SlotLayout(100_000_000, 8, 4,
                                                                       shares=tail_shares(4, 0.343, 3)).widths
    assert overlap_layout(80_000_000, 8).widths == SlotLayout(80_000_000, 8, 4, shares=tail_shares(4, 0.125)).widths
    assert overlap_layout(1000, 2, rounds=1).widths == SlotLayout(1000, 2, 1).widths


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fold(X, w, s=None, out=None, total=None, want_bf16=False, out_bf16=None):
    """engine.fold_stacked's contract, computed by the oracle (CPU ranks)."""
    from oracle import fedavg_oracle as O
    if X.dtype == torch.bfloat16:
        bits = np.ascontiguousarray(X.view(torch.int16).numpy()).view(np.uint16)
        f, b = O.fedavg_stacked_bf16(bits, w, s, total)
        res, resb = torch.from_numpy(f), torch.from_numpy(b.view(np.int16)).view(torch.bfloat16)
    else:
        res = torch.from_numpy(O.fedavg_stacked(np.ascontiguousarray(X.numpy()), w, s, total))
        resb = None
    if out is not None:
        out.copy_(res)
        res = out
    if out_bf16 is not None:
        out_bf16.copy_(resb)
        return out_bf16 if out is None else (res, out_bf16)
    return (res, resb) if want_bf16 else res


def _worker(rank, world, port, N, P, seed, scored, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agg = ShardedAggregator(fold=_oracle_fold)
        lo, hi = agg.bounds(P)
        X = torch.from_numpy(synth.clients_f32(seed, N, lo, hi - lo)) if hi > lo else torch.empty((N, 0))
        w = synth.cardinalities(seed, N)
        sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
        full = agg.aggregate(X, w, sc, P=P)
        q.put((rank, full.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P,scored", [(2, 10007, False), (2, 4096, True), (3, 130, False)])
def test_sharded_fold_gloo_matches_oracle(world, P, scored):
    from oracle import fedavg_oracle as O
    N, seed = 9, 17
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, P, seed, scored, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)] if scored else None
    exp = O.fedavg_stacked(X, w, sc)
    for r in range(world):
        out = np.frombuffer(got[r], dtype=np.float32)
        assert out.shape == exp.shape
        assert np.array_equal(out.view(np.uint32), exp.view(np.uint32)), r


def _slot_worker(rank, world, port, N, P, rounds, seed, q, tail=1.0, quantum=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agg = ShardedAggregator(fold=_oracle_fold)
        lay = SlotLayout(P, world, rounds, shares=tail_shares(rounds, tail), quantum=quantum)
        X = torch.zeros((N, lay.local_width))
        for k, (lo, hi) in enumerate(lay.slots(rank)):
            if hi > lo:
                o = lay.offset(k)
                X[:, o:o + hi - lo] = torch.from_numpy(synth.clients_f32(seed, N, lo, hi - lo))
        w = synth.cardinalities(seed, N)
        full = agg.aggregate_slots(X, w, None, lay)
        q.put((rank, full.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P,rounds,tail,quantum", [(2, 10007, 3, 1.0, 0), (3, 5000, 2, 1.0, 0),
                                                         (2, 64, 4, 1.0, 0), (2, 10007, 4, 0.25, 0),
                                                         (3, 20000, 3, 0.1, 0), (3, 20000, 4, 0.25, 1024)])
def test_overlapped_slot_gather_gloo_matches_oracle(world, P, rounds, tail, quantum):
    """Equal rounds, a short last round (tail_shares) and rounds in whole
    quanta reassemble the same model."""
    from oracle import fedavg_oracle as O
    N, seed = 7, 23
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slot_worker, args=(r, world, port, N, P, rounds, seed, q, tail, quantum))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = O.fedavg_stacked(synth.clients_f32(seed, N, 0, P), synth.cardinalities(seed, N))
    for r in range(world):
        out = np.frombuffer(got[r], dtype=np.float32)
        assert np.array_equal(out.view(np.uint32), exp.view(np.uint32)), r


def _step_form_worker(rank, world, port, cache, phase, N, P, rounds, seed, q):
    """phase "record": rank 0 records a step form (what "probe" does once it
    has measured); "restore": a fresh group of processes -- a later FaaS
    invocation -- runs its first aggregate_slots with one_launch="auto" and
    must find that form with no probe, no synchronisation and no collective
    besides the exchange's own all-gathers."""
    os.environ["FEDAVG_TUNE_CACHE"] = cache  # before the library is loaded in this process
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agg = ShardedAggregator(fold=_oracle_fold, device_ident="cputest:0")
        assert agg.one_launch == "auto"
        lay = SlotLayout(P, world, rounds, shares=tail_shares(rounds, 0.25))
        X = torch.zeros((N, lay.local_width))
        for k, (lo, hi) in enumerate(lay.slots(rank)):
            if hi > lo:
                X[:, lay.offset(k):lay.offset(k) + hi - lo] = torch.from_numpy(synth.clients_f32(seed, N, lo, hi - lo))
        w = synth.cardinalities(seed, N)
        if phase == "record":
            if rank == 0:
                agg.record_step_form(X, lay, one_launch=True)
            dist.barrier()
            q.put((rank, None))
            return
        used = []

        def forbid(name):
            def f(*a, **k):
                used.append(name)
                raise AssertionError(f"{name} called on the first aggregate_slots")
            return f
        real = {n: getattr(dist, n) for n in ("all_reduce", "broadcast", "barrier", "broadcast_object_list")}
        for n in real:
            setattr(dist, n, forbid(n))
        real_sync, real_event, real_probe = torch.cuda.synchronize, torch.cuda.Event, ShardedAggregator._record_probe
        torch.cuda.synchronize = forbid("torch.cuda.synchronize")
        torch.cuda.Event = forbid("torch.cuda.Event")
        ShardedAggregator._record_probe = forbid("probe")
        try:
            full = agg.aggregate_slots(X, w, None, lay)
            form = agg.step_form(X, lay)
        finally:
            for n, f in real.items():
                setattr(dist, n, f)
            torch.cuda.synchronize, torch.cuda.Event, ShardedAggregator._record_probe = real_sync, real_event, real_probe
        q.put((rank, (form, used, full.numpy().tobytes())))
    finally:
        dist.destroy_process_group()


def test_step_form_restored_in_a_new_process_without_probing(tmp_path):
    """The step-form choice outlives the process: a
    world-2 gloo group records it in the tuner's cache file; a second world-2
    group reads it on its first call with no probe call, no synchronize and
    no all_reduce, and still reassembles the oracle's model."""
    from oracle import fedavg_oracle as O
    N, P, rounds, seed, world = 11, 30011, 4, 29, 2
    cache = str(tmp_path / "tuner.txt")
    ctx = mp.get_context("spawn")
    for phase in ("record", "restore"):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_step_form_worker, args=(r, world, port, cache, phase, N, P, rounds, seed, q))
                 for r in range(world)]
        for p in procs:
            p.start()
        got = dict(q.get(timeout=120) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        if phase == "record":
            text = open(cache).read()
            assert text.count("fedavg-step ") == 1 and text.rstrip().endswith(" one"), text
    exp = O.fedavg_stacked(synth.clients_f32(seed, N, 0, P), synth.cardinalities(seed, N))
    for r in range(world):
        form, used, out = got[r]
        assert form == "one launch" and used == [], (r, form, used)
        assert np.array_equal(np.frombuffer(out, dtype=np.uint32), exp.view(np.uint32)), r


def _agree_worker(rank, world, port, cache, case, q):
    """Ranks with DIFFERENT cache files (another node, a concurrent writer):
    the first step of a shape takes rank 0's record on every rank."""
    os.environ["FEDAVG_TUNE_CACHE"] = cache
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lay = SlotLayout(40_000, world, 4)
        X = torch.zeros((9, lay.local_width))
        mine = {"both": [True, False, False][rank], "rank0_none": [None, True, False][rank]}[case]
        agg = ShardedAggregator(fold=_oracle_fold, device_ident="cputest:1")
        if mine is not None:
            agg.record_step_form(X, lay, one_launch=mine)
        fresh = ShardedAggregator(fold=_oracle_fold, device_ident="cputest:1")  # a later call's aggregator
        first = fresh._form(X, lay)
        again = fresh._form(X, lay)  # agreed once: no second collective (the group would hang if ranks differed)
        q.put((rank, (first, again, fresh.step_form(X, lay))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["both", "rank0_none"])
def test_step_form_is_rank0s_on_every_rank(tmp_path, case):
    """the step form is a group decision.  Rank 0 records
    one launch and ranks 1-2 per round (or rank 0 nothing): every rank runs
    rank 0's form, so none issues a collective the others do not."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, str(tmp_path / f"t{r}.txt"), case, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = (True, None) if case == "both" else (False, None)
    form = "one launch" if case == "both" else None
    for r in range(world):
        assert got[r] == (want, want, form), (r, got[r])


def test_probe_schedule_warms_times_then_decides(monkeypatch):
    """one_launch="probe" schedule (host logic, no GPU): the forms alternate,
    one launch first; each form's first PROBE_WARM calls are untimed (so a
    cold first call -- state, buffers, tuner -- cannot decide); the call that
    completes PROBE_STEPS compares the best timed call of each form, records
    the faster, and later calls run it without probing."""
    lay = SlotLayout(1000, 1, 4)
    agg = ShardedAggregator(one_launch="probe", device_ident="test:probe")
    monkeypatch.setattr(ShardedAggregator, "_lookup", lambda self, key: self._steps.get(key))
    rec = []
    monkeypatch.setattr(ShardedAggregator, "record_step_form",
                        lambda self, X, L, one: rec.append(one) or self._steps.__setitem__(self.step_key(X, L), one))

    class Ev:  # a timing event whose elapsed_time is the difference of fixed stamps
        def __init__(self, t):
            self.t = t

        def elapsed_time(self, other):
            return other.t - self.t

        def synchronize(self):
            pass

    X = torch.zeros(3, lay.local_width)
    # the one launch's warm call is slow (first use), its timed calls faster than per-round's
    times = {"one": [9.0, 1.0, 1.2], "per": [0.5, 1.1, 1.3]}
    seen = []
    for _ in range(ShardedAggregator.PROBE_STEPS):
        one, probing = agg._form(X, lay)
        form = "one" if one else "per"
        seen.append((form, probing[2]))
        t = times[form].pop(0)
        agg._record_probe(probing, *((Ev(0.0), Ev(t)) if probing[2] else (None, None)), X, lay)
    W, C = ShardedAggregator.PROBE_WARM, ShardedAggregator.PROBE_CALLS
    assert seen == [("one", False), ("per", False)] * W + [("one", True), ("per", True)] * C
    assert rec == [True]
    assert agg.probed[agg.step_key(X, lay)] == {"one": [1.0, 1.2], "per": [1.1, 1.3]}
    assert agg._form(X, lay) == (True, None)


def test_step_keys_and_modes():
    """The decision key names what the choice depends on; bad modes raise."""
    agg = ShardedAggregator(fold=_oracle_fold, device_ident="gfx950:256")
    lay = SlotLayout(100_000_000, 8, 4, shares=tail_shares(4, 0.343, 3))
    X = torch.zeros((200, lay.local_width), dtype=torch.bfloat16)
    key = agg.step_key(X, lay)
    assert key == f"gfx950:256 bf16 8 256 100000000 {','.join(map(str, lay.widths))}"
    assert ShardedAggregator(fold=_oracle_fold).step_key(X, lay) is None  # CPU tensor, no identity: no lookup
    with pytest.raises(ValueError):
        ShardedAggregator(one_launch="sometimes")
    with pytest.raises(ValueError):
        ShardedAggregator(check="later")


def _bf16_slot_worker(rank, world, port, N, P, rounds, seed, q, tail=1.0):
    """BASELINE config 4's layout in miniature: bf16 client rows in round-robin
    slots, fp32 fold per slot, RNE-bf16 slot outputs all-gathered (2 B/param)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agg = ShardedAggregator(fold=_oracle_fold)
        lay = SlotLayout(P, world, rounds, shares=tail_shares(rounds, tail))
        X = torch.zeros((N, lay.local_width), dtype=torch.int16)
        for k, (lo, hi) in enumerate(lay.slots(rank)):
            if hi > lo:
                X[:, lay.offset(k):lay.offset(k) + hi - lo] = torch.from_numpy(
                    synth.clients_bf16(seed, N, lo, hi - lo).view(np.int16))
        w = synth.cardinalities(seed, N)
        sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
        full = agg.aggregate_slots(X.view(torch.bfloat16), w, sc, lay)
        assert full.dtype == torch.bfloat16 and full.numel() == P
        q.put((rank, full.view(torch.int16).numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P,rounds,tail", [(2, 4099, 4, 1.0), (3, 1000, 2, 1.0), (2, 9000, 4, 0.25),
                                                  (8, 40011, 4, 0.343)])  # 8 ranks: the C4 exchange in miniature
def test_bf16_slot_gather_gloo_matches_oracle(world, P, rounds, tail):
    from oracle import fedavg_oracle as O
    N, seed = 6, 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bf16_slot_worker, args=(r, world, port, N, P, rounds, seed, q, tail))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    _, expb = O.fedavg_stacked_bf16(synth.clients_bf16(seed, N, 0, P), synth.cardinalities(seed, N), sc)
    for r in range(world):
        assert np.array_equal(np.frombuffer(got[r], dtype=np.uint16), expb), r


SHAPES = [(3, 5, 7), (64,), (33, 17), (1,), (900,)]


def _layers_worker(rank, world, port, N, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agg = ShardedAggregator(fold=_oracle_fold)
        P = sum(int(np.prod(s)) for s in SHAPES)
        X = synth.clients_f32(seed, N, 0, P)
        params = []
        for i in range(N):
            row, off = [], 0
            for shp in SHAPES:
                n = int(np.prod(shp))
                row.append(X[i, off:off + n].reshape(shp).copy())
                off += n
            params.append(row)
        w = synth.cardinalities(seed, N)
        sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)][: N - 2]  # zip() truncates to N-2 rows
        outs = agg.aggregate_layers(params, w, sc, device=torch.device("cpu"))
        q.put((rank, [o.tobytes() for o in outs], [o.shape for o in outs]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_aggregate_layers_slices_per_layer(world):
    """Reference-shaped per-layer lists through the sharded path: each rank
    copies only the layer pieces inside its bucket; zip() truncation keeps the
    divisor over every weight (stall_aware_aggregation.py:52-60)."""
    from oracle import fedavg_oracle as O
    N, seed = 7, 31
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layers_worker, args=(r, world, port, N, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, outs, shapes = q.get(timeout=120)
        got[r] = (outs, shapes)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    P = sum(int(np.prod(s)) for s in SHAPES)
    X = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)][: N - 2]
    exp = O.fedavg_stacked(X[: N - 2], w[: N - 2], sc, total=sum(w))
    for r in range(world):
        outs, shapes = got[r]
        assert [tuple(s) for s in shapes] == SHAPES
        flat = np.concatenate([np.frombuffer(b, dtype=np.float32) for b in outs])
        assert np.array_equal(flat.view(np.uint32), exp.view(np.uint32)), r


def test_aggregate_layers_rejects_other_dtypes():
    from fedlesscan_amd.aggregator.exceptions import InvalidParameterShapeError
    agg = ShardedAggregator(fold=_oracle_fold)
    with pytest.raises(InvalidParameterShapeError):
        agg.aggregate_layers([[np.zeros(4, np.float64)], [np.zeros(4, np.float64)]], [1, 2],
                             device=torch.device("cpu"))
    with pytest.raises(InvalidParameterShapeError):
        agg.aggregate_layers([[np.zeros(4, np.float32)], [np.zeros(4, np.float32)]], [np.float64(1), 2],
                             device=torch.device("cpu"))
