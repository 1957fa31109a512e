"""Host-side logic of the multi-GPU paths, no GPU needed:
  - the single-process drop-in's column partition (multigpu.py): buckets
    cover [0, P) exactly, are 64-element aligned, and the per-bucket layer
    views reassemble every row;
  - bench.py's rank launcher: `--gpus N` outside torch.distributed.run starts
    torch.distributed.run as a child with N ranks; a --gpus / WORLD_SIZE
    mismatch is a hard error.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("P", [0, 1, 63, 64, 65, 1000, 4097, 10_000_019])
@pytest.mark.parametrize("G", [1, 2, 3, 7, 8])
def test_column_buckets_partition(P, G):
    from fedlesscan_amd.multigpu import column_buckets
    b = column_buckets(P, G)
    assert len(b) == G
    assert b[0][0] == 0 and b[-1][1] == P
    for (lo, hi), (lo2, _) in zip(b, b[1:]):
        assert hi == lo2 and lo <= hi
    for lo, hi in b:
        assert lo % 64 == 0 or lo == P
    widths = [hi - lo for lo, hi in b if hi > lo]
    assert len(set(widths[:-1])) <= 1  # equal buckets, the last one short


def test_bucket_pieces_reassemble_rows():
    from fedlesscan_amd.multigpu import _bucket_pieces, _layer_offsets, column_buckets
    rng = np.random.default_rng(3)
    shapes = [(3, 5, 7), (11,), (), (1000, 3), (64,), (1,)]
    layers = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    flat = [np.ascontiguousarray(x).reshape(-1) for x in layers]
    offs = _layer_offsets(flat)
    P = int(offs[-1])
    row = np.concatenate(flat)
    for G in (1, 2, 3, 5, 8, 64):
        got = np.concatenate([np.concatenate(_bucket_pieces(flat, offs, lo, hi)) if hi > lo else
                              np.empty(0, np.float32) for lo, hi in column_buckets(P, G)])
        assert np.array_equal(got, row), G
        # pieces are views, never copies
        for lo, hi in column_buckets(P, G):
            for piece in _bucket_pieces(flat, offs, lo, hi):
                assert any(np.shares_memory(piece, f) for f in flat)


def test_resolve_devices():
    torch = pytest.importorskip("torch")
    from fedlesscan_amd.multigpu import resolve_devices
    assert resolve_devices([0, 1]) == [torch.device("cuda", 0), torch.device("cuda", 1)]
    assert resolve_devices("cuda:3") == [torch.device("cuda", 3)]
    assert resolve_devices(2) == [torch.device("cuda", 2)]
    assert resolve_devices([torch.device("cuda", 1), "cuda:0"]) == [torch.device("cuda", 1),
                                                                     torch.device("cuda", 0)]
    with pytest.raises(ValueError):
        resolve_devices(["cpu"])
    with pytest.raises(ValueError):
        resolve_devices([])


def _bench_env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                               "FEDAVG_BENCH_BACKEND")}
    env.update(kw)
    return env


def test_bench_gpus_mismatch_is_an_error():
    """Under a launcher, --gpus must equal WORLD_SIZE (no silent relabelling)."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_bench_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE 1" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_gpus_more_than_visible_is_an_error():
    """No GPU in this container: --gpus 2 outside a launcher refuses before
    starting anything (no 1-GPU line labelled n_gpus 2)."""
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_bench_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_launches_torch_distributed_run_as_child(monkeypatch):
    """--gpus N > 1 outside torch.distributed.run: the child command is
    torch.distributed.run with N ranks on 127.0.0.1 running bench.py with the
    same arguments, and its exit status is returned."""
    sys.path.insert(0, REPO)
    import bench
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("FEDAVG_BENCH_BACKEND", "gloo")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--config", "c4", "--steps", "3"])
    args = bench.parse()
    assert bench.launch_ranks(args) == 7
    cmd = seen["cmd"]
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m"
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[-7:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--config", "c4", "--steps", "3"]
    # a rank itself (WORLD_SIZE set) or one GPU: no launch
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.launch_ranks(args) is None
    monkeypatch.delenv("WORLD_SIZE")
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.launch_ranks(bench.parse()) is None


def test_bench_default_slot_layouts():
    """bench.DEFAULT_TAIL: for every world size of the scaling run, the default
    per-dtype slot layouts of C3 (weak: 10M params per rank) and C4 (strong:
    100M in total) cover the model, stay 64-aligned, and shrink toward the
    last round (whose all-gather is the one left exposed)."""
    sys.path.insert(0, REPO)
    import bench
    from fedlesscan_amd.sharding import SlotLayout, tail_shares
    for world in (1, 2, 4, 8):
        for cfg in ("c3", "c4"):
            N, P, dt = bench.CONFIGS[cfg][:3]
            P_total = P * world if bench.CONFIGS[cfg][6] == "weak" else P
            tail, steps = bench.DEFAULT_TAIL[dt]
            lay = SlotLayout(P_total, world, 4, shares=tail_shares(4, tail, steps))
            assert lay.padded_total >= P_total and lay.padded_total - P_total < 64 * world * 4 + 64 * world
            assert all(w % 64 == 0 for w in lay.widths)
            assert lay.widths == sorted(lay.widths, reverse=True) and lay.widths[-1] < lay.widths[0]
            assert abs(lay.widths[-1] / lay.widths[0] - tail) < 0.01
            covered = sorted(sl for r in range(world) for sl in lay.slots(r) if sl[1] > sl[0])
            assert covered[0][0] == 0 and covered[-1][1] == P_total
            assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


def test_bench_step_mode_flags(monkeypatch):
    """--step-mode auto (default) / one / per-round; --per-round-launches is
    per-round; --warmup-s defaults to exactly W warm-up steps."""
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.step_mode == "auto" and not a.per_round_launches and a.warmup_s == 0.0
    monkeypatch.setattr(sys, "argv", ["bench.py", "--step-mode", "one", "--warmup-s", "1.5"])
    a = bench.parse()
    assert a.step_mode == "one" and a.warmup_s == 1.5
    monkeypatch.setattr(sys, "argv", ["bench.py", "--per-round-launches"])
    assert bench.parse().per_round_launches
    monkeypatch.setattr(sys, "argv", ["bench.py", "--step-mode", "sometimes"])
    with pytest.raises(SystemExit):
        bench.parse()


def test_model_digest_separates_models():
    """gather_check's digests: the same bits give the same pair on every rank
    (chunking and reduction order do not change them); a flipped bit, two
    swapped elements or a shifted slot give another pair."""
    import torch

    import bench
    g = torch.Generator().manual_seed(5)
    for dt in (torch.int32, torch.int16):
        bits = torch.randint(-(1 << 15), 1 << 15, (100_003,), generator=g).to(dt)
        d = bench.model_digest(bits)
        assert torch.equal(d, bench.model_digest(bits.clone(), chunk=4099))
        flipped = bits.clone()
        flipped[777] ^= 1
        swapped = bits.clone()
        swapped[[10, 90_000]] = bits[[90_000, 10]]
        shifted = torch.roll(bits, 64)
        for other in (flipped, swapped, shifted):
            assert not torch.equal(d, bench.model_digest(other))
