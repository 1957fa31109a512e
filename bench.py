#!/usr/bin/env python3
"""Headline benchmark: device-resident N-client FedAvg fp32 reduction (aggregated GB/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5|c4] [--variant V]
                    [--sweep] [--no-cpu-baseline]

One "step" = one aggregation round over one batch already resident in HBM:
the fa_fedavg_f32 fold of [N_clients x P] -> [P] (stall-aware for c5, bf16 for
c4), plus, at world size > 1, the RCCL all-gather of every rank's output
bucket over xGMI (the one real exchange step of the path: SURVEY 8e).

Default workload = BASELINE config 3: 1024 clients x 10,000,000 fp32 params on
ONE GPU.  With --gpus N (one process per GPU) every rank owns its own
10M-param bucket of a 10M*N-param model (weak scaling) and the global model is
reassembled by all_gather_into_tensor (RCCL over xGMI).  `python bench.py
--gpus N` with N > 1 outside torch.distributed.run starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py ...` as a
child process (before anything touches the GPU), passes its output through and
exits with its status; under torch.distributed.run, --gpus must equal
WORLD_SIZE.  Under torch.distributed.run the process group is initialised even
at WORLD_SIZE 1 (nccl = RCCL), so the gather path runs on real RCCL streams.

Inputs: integer-exact synthetic generator (fedlesscan_amd/synth.py), generated
directly in HBM by fa_synth_*; random-init, no dataset.  Rank 0 at N=1 also
times the CPU oracle on a bounded column sample of the same workload and
checks the GPU output on that sample bit-for-bit.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from fedlesscan_amd import _lib, synth  # noqa: E402
from fedlesscan_amd.engine import Factors  # noqa: E402
from fedlesscan_amd.sharding import ALIGN, DEFAULT_TAIL, SlotLayout, gather_into, tail_shares  # noqa: E402
from fedlesscan_amd.sharding import fold_stream as sharding_fold_stream  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (clients, params, dtype, scored, seed, card_hi, scaling, description)
    #   scaling "weak":   `params` per GPU, the model grows with the GPU count
    #   scaling "strong": `params` in total, split into per-GPU buckets
    "c2": (100, 1_000_000, "f32", False, 2, 600, "weak",
           "100 clients x 1M fp32 FedAvg, 1 MI355X (BASELINE config 2)"),
    "c3": (1024, 10_000_000, "f32", False, 3, 600, "weak",
           "1024 clients x 10M fp32 FedAvg per GPU, device-resident (BASELINE config 3, headline)"),
    "c4": (256, 100_000_000, "bf16", False, 4, 600, "strong",
           "256 clients x 100M bf16, parameter buckets over the GPUs + RCCL gather (BASELINE config 4)"),
    "c5": (512, 25_000_000, "f32", True, 5, 2000, "weak",
           "512 clients x 25M fp32 FedLesScan stall-aware, tolerance 2, R=10 (BASELINE config 5)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-s", type=float, default=0.0,
                    help="after the W warm-up steps, more untimed steps until about this many seconds of warm-up "
                         "have run (the same count on every rank); 0 (default) = exactly W.  Measured A/B on one "
                         "box: C3 unchanged (7060-7068 GB/s either way), C2 slower after 10,000 extra launches "
                         "(5.7-6.2 TB/s against 6.7-6.8; profiles/r04_warmup_ab.log)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--sweep", action="store_true", help="time every kernel variant (stderr table)")
    ap.add_argument("--variants", default="", help="with --sweep: comma-separated variant numbers only")
    ap.add_argument("--splitn", action="store_true",
                    help="time the opt-in split-client fold (fa_fedavg_f32_splitn, NOT bit-exact) instead")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-lean", action="store_true",
                    help="skip the full-size one-core reference timing (cpu_baseline.full_lean)")
    ap.add_argument("--unpadded", action="store_true",
                    help="row pitch = the model size exactly (experiments: odd sizes give rows that are not 16-B "
                         "aligned, as a torch.stack of such a model)")
    ap.add_argument("--pitch-extra", type=int, default=0,
                    help="extra row padding in elements on top of the layout's (row-pitch experiments)")
    ap.add_argument("--cpu-cols", type=int, default=1 << 21, help="columns in the CPU baseline sample")
    ap.add_argument("--cpu-reps", type=int, default=8)
    ap.add_argument("--clients", type=int, default=0, help="override the config's client count (experiments)")
    ap.add_argument("--params", type=int, default=0, help="override the config's parameter count (experiments)")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="initialise a one-rank nccl (RCCL) process group in this process, without a launcher, so the "
                         "all-gather path runs under a profiler that must start the program itself (one GPU)")
    ap.add_argument("--rounds", type=int, default=0,
                    help="exchange rounds per step (fold of round k+1 overlaps the all-gather of round k); "
                         "default 1 on one GPU, 4 on several")
    ap.add_argument("--tail", type=float, default=None,
                    help="last exchange round's slot as a fraction of the others' (its all-gather is the one "
                         "left exposed after the step's folds); 1 = equal rounds.  Default with several rounds: "
                         "the layout for the dtype (DEFAULT_TAIL)")
    ap.add_argument("--step-mode", default="auto", choices=["auto", "probe", "one", "per-round"],
                    help="with several rounds under a process group: 'one' = the whole step in one fold launch, "
                         "each round's all-gather started behind its completion flag; 'per-round' = one fold "
                         "launch per exchange round (round 3's step); 'probe' = time both on this run's own "
                         "ranks before the warm-up (max over ranks, best of two trials), keep the faster and "
                         "record it in the tuner's cache file (fa_step_record); 'auto' (default) = the form "
                         "recorded for this machine and shape (rank 0's record), or 'probe' when none is")
    ap.add_argument("--per-round-launches", action="store_true", help="same as --step-mode per-round")
    ap.add_argument("--exchange", default="rccl", choices=["rccl", "peer_copy"],
                    help="the one-launch step's exchange: 'rccl' = an all_gather_into_tensor per round behind its "
                         "wait; 'peer_copy' = copy-engine pulls of the peers' slots through IPC-opened buffers "
                         "(sharding.PeerExchange, fa_peers); the gathered model is checked against an RCCL step's")
    ap.add_argument("--step-impl", default="product", choices=["product", "loop"],
                    help="under a process group: 'product' (default) = every step is one call of the shipped "
                         "ShardedAggregator.aggregate_slots (sharding.py; --step-mode and --exchange map onto its "
                         "one_launch and exchange, --check onto its check); 'loop' = this file's own step loop "
                         "over the same library calls, for comparison")
    ap.add_argument("--check", default="sync", choices=["sync", "deferred"],
                    help="--step-impl product: ShardedAggregator's round-wait check, 'sync' (its default: every "
                         "call waits for its waits and agrees over the ranks) or 'deferred' (one check_timeouts() "
                         "after the K timed steps, inside the timed region)")
    ap.add_argument("--tail-steps", type=int, default=None,
                    help="rounds over which the slots shrink geometrically to --tail (2 with --tail 0.25 and 4 "
                         "rounds: shares 1, 1, 0.5, 0.25)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N > 1 run without torch.distributed.run: start it as a CHILD
    process with one rank per GPU and return its exit status (None: this
    process is a rank itself).  Runs before anything initialises the GPU (no
    exec from a process that has: the child is a separate process), so the
    N-GPU line is always N real ranks, never a relabelled 1-GPU run."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    if os.environ.get("FEDAVG_BENCH_BACKEND") != "gloo":
        # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if args.gpus > have:
            log(f"error: --gpus {args.gpus} but only {have} GPU(s) visible "
                "(FEDAVG_BENCH_BACKEND=gloo rehearses more ranks than GPUs)")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    log("launching " + " ".join(cmd))
    return subprocess.call(cmd)  # rank 0's JSON line reaches our stdout unchanged


def setup_dist(args):
    """(world, rank, device, backend).  Under torch.distributed.run the process
    group is initialised at any world size, WORLD_SIZE 1 included, so the
    all-gather path always runs (nccl = RCCL over xGMI)."""
    if getattr(args, "rccl_world1", False) and "WORLD_SIZE" not in os.environ:
        if args.gpus != 1:
            raise SystemExit("bench.py: --rccl-world1 runs one rank (--gpus 1)")
        os.environ.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(_free_port()))
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: the line would not measure "
                         f"{args.gpus} GPUs")
    backend = None
    if launched:
        if os.environ.get("FEDAVG_BENCH_BACKEND") == "gloo":
            # rehearsal on a box with fewer GPUs than ranks: ranks share devices,
            # the gather goes through gloo (host memory); never a headline number
            torch.cuda.set_device(local % torch.cuda.device_count())
            backend = "gloo"
            dist.init_process_group(backend)
        else:
            torch.cuda.set_device(local)
            backend = "nccl"
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", torch.cuda.current_device()), backend


def json_stdout():
    """A writer on the real stdout for the one JSON line; fd 1 itself is
    pointed at stderr for the rest of the run, because RCCL prints its version
    banner (and the HIP runtime its notices) on stdout, which would put extra
    lines before the JSON line of a multi-GPU run."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(real, "w")


def rank_devices(dev) -> list:
    """Every rank's GPU (rank order): ordinal and PCI bus id."""
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": dist.get_rank() if dist.is_initialized() else 0, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "device": dev.index, "pci_bus_id": getattr(props, "pci_bus_id", None),
          "pci_device_id": getattr(props, "pci_device_id", None), "name": props.name}
    if not dist.is_initialized():
        return [me]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def model_digest(bits: torch.Tensor, chunk: int = 1 << 24) -> torch.Tensor:
    """Two int64 digests of a model's bit patterns (an int16 or int32 view):
    their sum and a position-weighted sum (weights 1..1021, cycling), both
    modulo 2^64 -- integer sums wrap, so the order of the reduction does not
    matter and every rank computes the same digests for the same bits.  Used
    by gather_check: equal digests on every rank = one model on every rank."""
    mask = (1 << (8 * bits.element_size())) - 1
    flat = bits.reshape(-1)
    s = torch.zeros(2, dtype=torch.int64, device=bits.device)
    for lo in range(0, flat.numel(), chunk):
        x = flat[lo:lo + chunk].to(torch.int64) & mask
        w = torch.arange(lo, lo + x.numel(), dtype=torch.int64, device=bits.device) % 1021 + 1
        s[0] += x.sum()
        s[1] += (x * w).sum()
    return s


class Workload:
    """This rank's share of the synthetic round: its parameter slots, all clients.

    The global model is cut by SlotLayout into rounds*world slots; rank r owns
    slots k*world + r (k < rounds), stored side by side in X [N, rounds*sub].
    With rounds=1 that is one contiguous bucket per rank."""

    def __init__(self, cfg, rank, world, dev, rounds, align=None, pitch_extra=0, tail=1.0, tail_steps=1,
                 exchange_step=False):
        self.N, P, self.dtype, self.scored, self.seed, card_hi, self.scaling, self.desc = cfg
        self.P_total = P * world if self.scaling == "weak" else P
        self.layout = SlotLayout(self.P_total, world, rounds, align=ALIGN if align is None else align,
                                 shares=tail_shares(rounds, tail, tail_steps))
        self.slots = self.layout.slots(rank)
        self.P = sum(hi - lo for lo, hi in self.slots)  # real columns this rank folds
        self.rank, self.world, self.dev = rank, world, dev
        B = _lib.load_bench()  # input generator (bench / test support library)
        st = torch.cuda.current_stream(dev).cuda_stream
        tdt = torch.float32 if self.dtype == "f32" else torch.bfloat16
        W = self.layout.local_width
        self.ldx = W + pitch_extra  # row pitch (elements): the slots side by side, plus any extra padding
        self.X = torch.zeros((self.N, self.ldx), dtype=tdt, device=dev)
        gen = B.fa_synth_f32 if self.dtype == "f32" else B.fa_synth_bf16
        esz = self.X.element_size()
        for k, (lo, hi) in enumerate(self.slots):
            if hi > lo:
                _lib.check(gen(self.X.data_ptr() + self.layout.offset(k) * esz, self.N, hi - lo, self.ldx, self.seed, 0, lo, st),
                           "synth", bench=True)
        self.col0 = self.slots[0][0]
        self.weights = synth.cardinalities(self.seed, self.N, 1, card_hi)
        self.scores = ([(r + 1) / 11 for r in synth.round_ids(self.seed, self.N, 10, 2)]
                       if self.scored else None)
        f = Factors(self.weights, self.scores, np.dtype(np.float32))
        self.a, self.s = f.to(dev)
        self.div = float(f.div)
        self.out = torch.empty(W, dtype=torch.float32, device=dev)  # this rank's slots, side by side
        # bf16 models also write the RNE bf16 copy of the result (the form the
        # multi-GPU gather moves: half the xGMI bytes of the fp32 result)
        self.out_bf16 = torch.empty(W, dtype=torch.bfloat16, device=dev) if self.dtype == "bf16" else None
        # an exchange step of bf16 rows stores only the bf16 copy it exchanges
        # (ABI 5: no fp32 result, as ShardedAggregator); one GPU alone writes both
        self.write_f32 = not (exchange_step and self.dtype == "bf16")
        elt = 4 if self.dtype == "f32" else 2
        # algorithmic bytes per step on this rank: every real input element once + each output written once
        # (fp32 4 B, the bf16 copy 2 B per param)
        self.bytes = (self.N * self.P * elt + (self.P * 4 if self.write_f32 else 0)
                      + (self.P * 2 if self.dtype == "bf16" else 0))
        torch.cuda.synchronize()

    def launch(self, variant=0, k=0):
        """Fold round k's slot (all of X when rounds == 1).  variant 0 is the
        product entry point (fa_fedavg_f32 / fa_fedavg_bf16 of libfedavg_hip.so);
        others come from the tuning library."""
        L = _lib.load()
        st = torch.cuda.current_stream(self.dev).cuda_stream
        s = None if self.s is None else self.s.data_ptr()
        off, sub = self.layout.offset(k), self.layout.width(k)
        x = self.X.data_ptr() + off * self.X.element_size()
        o = self.out.data_ptr() + off * 4 if self.write_f32 else None
        ob = None if self.out_bf16 is None else self.out_bf16.data_ptr() + off * 2
        bench = variant > 0
        if self.dtype == "f32" and variant < 0:  # opt-in split-client fold
            rc = L.fa_fedavg_f32_splitn(x, self.N, sub, self.ldx, self.a.data_ptr(), s, self.div, o, st)
        elif self.dtype == "f32" and variant == 0:
            rc = L.fa_fedavg_f32(x, self.N, sub, self.ldx, self.a.data_ptr(), s, self.div, o, st)
        elif self.dtype == "f32":
            rc = _lib.load_bench().fa_fedavg_f32_variant(x, self.N, sub, self.ldx, self.a.data_ptr(), s, self.div, o, st,
                                                         variant)
        elif variant == 0:
            rc = L.fa_fedavg_bf16(x, self.N, sub, self.ldx, self.a.data_ptr(), s, self.div, o, ob, st)
        else:
            rc = _lib.load_bench().fa_fedavg_bf16_variant(x, self.N, sub, self.ldx, self.a.data_ptr(), s, self.div, o,
                                                          ob, st, variant)
        if rc:
            _lib.check(rc, "fold", bench=bench)


def cpu_baseline(wl: Workload, ncols: int, reps: int = 3):
    """Oracle on host cores over a bounded column sample of the same workload
    (rank 0's first slot: the GPU output of those columns is checked bit for
    bit against it)."""
    from oracle import fedavg_oracle as O  # checker / CPU baseline only
    from oracle import oracle_lib as OL
    ncols = min(ncols, wl.slots[0][1] - wl.slots[0][0])
    t0 = time.time()
    Xh = OL.synth_f32(wl.seed, wl.N, ncols, col0=wl.col0) if wl.dtype == "f32" else \
        synth.bf16_bits_to_f32(OL.synth_bf16(wl.seed, wl.N, ncols, col0=wl.col0))
    gen_s = time.time() - t0
    sample_bytes = wl.N * ncols * (4 if wl.dtype == "f32" else 2) + ncols * 4
    # (i) literal numpy restatement of fed_avg_aggregator.py:24-42 (1 core: numpy ufuncs are single-threaded)
    params = [[Xh[i]] for i in range(wl.N)]
    t_np_all = []
    for _ in range(max(1, reps)):
        t0 = time.perf_counter()
        if wl.scored:
            ref = O.stall_aware_literal([{"round_id": r} for r in synth.round_ids(wl.seed, wl.N, 10, 2)], 10,
                                        params, wl.weights)[0]
        else:
            ref = O.fedavg_literal(params, wl.weights)[0]
        t_np_all.append(time.perf_counter() - t0)
    t_np = sorted(t_np_all)[len(t_np_all) // 2]
    del params
    # (ii) bit-identical C restatement, OpenMP over all host cores
    threads = OL.max_threads()
    a = np.array(wl.weights, np.float32)
    s = None if wl.scores is None else np.array(wl.scores, np.float32)
    t_omp = []
    for _ in range(3):
        t0 = time.perf_counter()
        ref_omp = OL.fedavg_f32(Xh, a, np.float32(wl.div), s=s, nthreads=threads)
        t_omp.append(time.perf_counter() - t0)
    if wl.write_f32:
        gpu_same = np.array_equal(wl.out[:ncols].cpu().numpy().view(np.uint32), ref.view(np.uint32))
    else:  # a bf16 exchange step stores only the RNE-bf16 copy of the result
        gpu_same = np.array_equal(wl.out_bf16[:ncols].view(torch.int16).cpu().numpy().view(np.uint16),
                                  synth.f32_to_bf16_bits(ref))
    exact = bool(gpu_same and np.array_equal(ref_omp.view(np.uint32), ref.view(np.uint32)))
    visible = len(os.sched_getaffinity(0))
    return {
        "value": round(sample_bytes / t_np / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
        "form": "literal: every client's `layer * n` product kept, then reduce(np.add) and one divide "
                "(fed_avg_aggregator.py:31-41), on a column sample (the full workload: full_lean)",
        "sample": f"{wl.N} clients x first {ncols} params of the same workload (rank 0's first slot, columns "
                  f"{wl.col0}..{wl.col0 + ncols}); numpy literal restatement of fed_avg_aggregator.py:24-42 "
                  f"(1 core, numpy ufuncs single-threaded), median of {len(t_np_all)} runs {t_np:.2f} s "
                  f"(total {sum(t_np_all):.1f} s)",
        "sample_temporaries": f"each `layer * n` product is a fresh {ncols * 4 / 1e6:.1f} MB float32 array "
                              f"(the full workload's rows are {wl.P * 4 / 1e6:.1f} MB): the sample is friendlier "
                              "to the caches than the whole job, so this rate is an upper bound for the "
                              "reference on the full workload",
        "omp": {"value": round(sample_bytes / min(t_omp) / 1e9, 3), "unit": "GB/s", "cores": threads,
                "kind": "port", "impl": "oracle/fedavg_ref.c (bit-identical, OpenMP)",
                "cores_note": f"{threads} OpenMP threads of the {visible} CPUs visible: OMP_NUM_THREADS "
                              f"({os.environ.get('OMP_NUM_THREADS', 'unset')}) is the host CPU share of one GPU "
                              "on the GPU box; the other visible CPUs belong to the node's other GPUs"},
        "host_cpus_visible": visible,
        "sample_bit_exact_vs_gpu": exact,
        "gen_s": round(gen_s, 2),
    }


def cpu_full_lean(wl: Workload):
    """The reference algorithm over the WHOLE workload on one core (SURVEY 8(d):
    "time the lean form at full size"): the inputs copied from HBM to host
    memory (not timed), then oracle.fedavg_stacked -- the op order of
    fed_avg_aggregator.py:31-41 / stall_aware_aggregation.py:55-66 with one
    product temporary instead of N (np.multiply into a [P] buffer, np.add into
    the running sum, one true_divide; bit-identical to the literal form) --
    and every output column compared with the GPU's.  fp32 workloads at one
    rank's single slot only (N = 1 GPU, rounds = 1)."""
    from oracle import fedavg_oracle as O  # CPU baseline / checker only
    if wl.dtype != "f32" or len(wl.slots) != 1:
        return None
    t0 = time.perf_counter()
    Xh = torch.empty((wl.N, wl.ldx), dtype=torch.float32)
    Xh.copy_(wl.X)
    d2h_s = time.perf_counter() - t0
    Xn = Xh.numpy()[:, :wl.P]
    t0 = time.perf_counter()
    ref = O.fedavg_stacked(Xn, wl.weights, wl.scores)
    t = time.perf_counter() - t0
    exact = bool(np.array_equal(ref.view(np.uint32), wl.out[:wl.P].cpu().numpy().view(np.uint32)))
    nbytes = wl.N * wl.P * 4 + wl.P * 4
    del Xh, Xn
    return {"value": round(nbytes / t / 1e9, 3), "unit": "GB/s", "seconds": round(t, 2), "bytes": nbytes,
            "cores": 1, "kind": "port",
            "impl": "oracle.fedavg_stacked: the reference op order over the full workload with one [P] product "
                    "temporary (numpy ufuncs, single-threaded)",
            "d2h_s": round(d2h_s, 2), "bit_exact_vs_gpu_all_columns": exact}


def read_traffic(config: str):
    """PMC HBM bytes per launch from the committed rocprofv3 --pmc passes
    (profiles/pmc_<config>.json, written by scripts/profile_c3.sh): counters
    cannot be read from inside the timed run, so the line names that pass."""
    p = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    src = os.path.relpath(p, REPO)
    if d.get("provenance"):
        src += f" ({d['provenance']})"
    return d.get("hbm_bytes_per_launch"), src


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    out = json_stdout()
    world, rank, dev, backend = setup_dist(args)
    dist_on = dist.is_initialized()  # every rank-collective branch below keys on this, not on world > 1
    cfg = CONFIGS[args.config]
    if args.clients or args.params:
        cfg = (args.clients or cfg[0], args.params or cfg[1], *cfg[2:7],
               cfg[7] + f" [override: {args.clients or cfg[0]} clients x {args.params or cfg[1]} params]")
    rounds = args.rounds or (4 if dist_on else 1)
    if args.splitn:
        args.variant = -1
    wl = Workload(cfg, rank, world, dev, rounds, align=1 if args.unpadded else None, pitch_extra=args.pitch_extra,
                  tail=(args.tail if args.tail is not None else DEFAULT_TAIL[cfg[2]][0]) if rounds > 1 else 1.0,
                  tail_steps=args.tail_steps if args.tail_steps is not None else DEFAULT_TAIL[cfg[2]][1],
                  exchange_step=dist_on)
    # the shipped class steps the multi-GPU run (a sweep or a split fold times this file's own launches)
    product = dist_on and args.step_impl == "product" and args.variant == 0 and not args.sweep
    B = _lib.load_bench()
    lay = wl.layout
    full = torch.empty(lay.padded_total, dtype=torch.float32 if wl.dtype == "f32" else torch.bfloat16,
                       device=dev) if dist_on else None
    stream = torch.cuda.current_stream(dev)
    if dist_on:
        # the folds on a high-priority stream: HIP maps streams onto a few
        # hardware queues, and a fold sharing one with RCCL's stream queues
        # behind the previous round's collective instead of overlapping it
        # (profiles/r03_c4_trace/: fold k+1 started ~35 us after fold k, behind
        # the all-gather's copy, when both sat on one queue)
        stream = sharding_fold_stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))

    # the library's tuner times each candidate kernel form on the first calls of
    # a new shape (fa_set_autotune): run the folds alone (no collectives, so the
    # ranks need not agree on a count) until every slot shape has its form, as
    # the first aggregation rounds of a deployment would
    L = _lib.load()
    tune_calls = 0
    step_mode = "per-round" if args.per_round_launches else args.step_mode
    can_one = dist_on and rounds > 1 and args.variant == 0 and step_mode != "per-round"
    # "auto": the step form recorded for this machine and shape (the product's
    # ShardedAggregator reads the same record), or, with none, both forms timed
    # below and the faster recorded; "probe": time them whatever is recorded
    from fedlesscan_amd.sharding import device_ident, step_key as make_step_key
    skey = make_step_key(device_ident(dev), wl.dtype == "bf16", wl.N, lay, args.exchange) if can_one else None
    recorded = L.fa_step_lookup(skey.encode()) if (can_one and step_mode == "auto") else -1
    if can_one and world > 1:  # every rank runs rank 0's record (ranks may share no cache file)
        t = torch.tensor([recorded], dtype=torch.int64, device=dev)
        dist.broadcast(t, src=0)
        recorded = int(t.item())
    # the product's own probe (ShardedAggregator one_launch="probe") decides during the warm-up
    probe_modes = can_one and step_mode in ("auto", "probe") and recorded < 0 and not product
    one_launch = can_one and (recorded != 0)
    per_round_possible = not can_one or probe_modes or (product and step_mode != "one")
    if args.variant == 0 and L.fa_set_autotune(-1) == 1 and per_round_possible:
        for tune_calls in range(1, 201):
            for k in range(rounds):
                wl.launch(0, k)
            torch.cuda.synchronize()
            if L.fa_autotune_pending() == 0:
                break

    # every rank runs rank 0's measured forms (the tuner measures per process:
    # ranks could otherwise fold the same slot shape with different kernels);
    # what each rank had chosen on its own is reported
    forms_by_rank, forms_agree = None, None
    if dist_on and world > 1 and args.variant == 0:
        kind = 1 if wl.dtype == "f32" else 2
        mine = {}
        if can_one:  # one fixed step form per dtype
            mine["step"] = L.fa_rounds_form(1 if wl.dtype == "bf16" else 0).decode()
        if per_round_possible:
            mine.update({str(w): L.fa_fold_form(kind, wl.N, w, wl.ldx, 1 if wl.scored else 0,
                                                stream.cuda_stream).decode() for w in dict.fromkeys(lay.widths)})
        forms_by_rank = [None] * world
        dist.all_gather_object(forms_by_rank, mine)
        forms_agree = all(f == forms_by_rank[0] for f in forms_by_rank)
        if per_round_possible:
            text = [_lib.tune_export() if rank == 0 else None]
            dist.broadcast_object_list(text, src=0)
            if rank != 0:
                _lib.tune_import(text[0])

    if args.sweep and rank == 0:
        nvar = B.fa_num_variants() if wl.dtype == "f32" else B.fa_num_bf16_variants()
        vname = B.fa_variant_name if wl.dtype == "f32" else B.fa_bf16_variant_name
        chosen = [int(x) for x in args.variants.split(",") if x] or list(range(nvar))
        res = {v: [] for v in chosen}
        for _ in range(2):
            for v in chosen:
                wl.launch(v)
        order = list(chosen)
        rng = np.random.default_rng(12345)
        # back-to-back launches of one variant between two events: per-launch
        # events would add a few microseconds to every small-model launch
        batch = max(1, min(20, int(2e9 // max(wl.bytes, 1))))
        for _ in range(max(args.steps, 5)):
            rng.shuffle(order)  # a fresh order each round: no variant always runs first
            for v in order:  # interleaved rounds in one process
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _b in range(batch):
                    for k in range(rounds):
                        wl.launch(v, k)
                e1.record(stream)
                e1.synchronize()
                res[v].append(e0.elapsed_time(e1) / batch)
        for v, ts in res.items():
            ts = sorted(ts)
            log(f"variant {v} {vname(v).decode():10s} median {ts[len(ts)//2]:.4f} ms  "
                f"min {ts[0]:.4f} ms  -> {wl.bytes / (ts[len(ts)//2] * 1e-3) / 1e9:.1f} GB/s")

    # the exchanged model: fp32 result for fp32 updates, the RNE bf16 result
    # for bf16 updates (2 B/param over xGMI: half the bytes of the fp32 result)
    send = wl.out if wl.dtype == "f32" else wl.out_bf16
    if can_one:
        from fedlesscan_amd import engine
        from fedlesscan_amd.sharding import gather_stream
        gs = gather_stream(dev)
        offs = [lay.offset(k) for k in range(rounds + 1)]

    px = None
    agg = None
    if product:
        from fedlesscan_amd.sharding import ShardedAggregator
        ol = {"auto": "probe", "probe": "probe", "one": True, "per-round": False}[step_mode] if can_one else False
        agg = ShardedAggregator(one_launch=ol, exchange=args.exchange, check=args.check)
    elif can_one and args.exchange == "peer_copy":
        from fedlesscan_amd.sharding import PeerExchange
        px = PeerExchange(None, dev, lay, wl.dtype == "bf16")

    def step_one_launch(ev=None, exchange=None):
        """The whole step in one fold launch; round k's all-gather on the gather
        stream behind a wait for round k's completion flag (mid-launch), or the
        peer copy (--exchange peer_copy)."""
        if (exchange or args.exchange) == "peer_copy":
            if ev is not None:
                ev[0][0][0].record(stream)
            px.step(wl.X, wl.weights, wl.scores, full, None, stream, gs)
            if ev is not None:
                ev[0][0][1].record(stream)
            stream.wait_stream(gs)
            if ev is not None:
                ev[1].record(stream)
            return
        if ev is not None:
            ev[0][0][0].record(stream)
        r = engine.fold_rounds(wl.X, wl.weights, wl.scores, offs, out=wl.out if wl.write_f32 else None,
                               out_bf16=wl.out_bf16)
        if ev is not None:
            ev[0][0][1].record(stream)
        works = []
        for k in range(rounds):
            engine.wait_round(r, k, gs)
            lo, hi = lay.round_range(k)
            with torch.cuda.stream(gs):
                w = gather_into(full[lo:hi], send[lay.offset(k):lay.offset(k + 1)], None, async_op=True)
            if w is not None:
                works.append(w)
        for w in works:
            w.wait()  # the fold stream waits for the RCCL stream
        stream.wait_stream(gs)
        if ev is not None:
            ev[1].record(stream)

    def step(ev=None, mode=None):
        """ev = (fold events per round, end event) for the timed steps; mode
        "one" / "per-round" overrides the chosen step form (the probe).  The
        product: one aggregate_slots call (its own events: agg.trace)."""
        if product:
            agg.aggregate_slots(wl.X, wl.weights, wl.scores, lay, out=full)
            return
        if (one_launch if mode is None else mode == "one"):
            step_one_launch(ev)
            return
        works = []
        for k in range(rounds):
            if ev is not None:
                ev[0][k][0].record(stream)
            wl.launch(args.variant, k)
            if ev is not None:
                ev[0][k][1].record(stream)
            if dist_on:  # reassemble the global model: RCCL all-gather over xGMI, overlapping round k+1
                lo, hi = lay.round_range(k)
                w = gather_into(full[lo:hi], send[lay.offset(k):lay.offset(k + 1)], None, async_op=True)
                if w is not None:
                    works.append(w)
        for w in works:
            w.wait()  # the compute stream waits for the RCCL stream
        if ev is not None:
            ev[1].record(stream)

    if product:
        # the caller's stream is the default stream: aggregate_slots moves its
        # folds onto the high-priority fold stream itself and joins back
        stream = torch.cuda.current_stream(dev)
    else:
        torch.cuda.set_stream(stream)  # the folds and the collectives' waits run on `stream` from here on
    mode_probe = None
    if probe_modes:
        # which step form is faster depends on how much the exchange kernels
        # slow the fold, which only this run's own ranks and links can tell
        # (DESIGN §8): time both, every rank in step, before the warm-up
        modes = ("one", "per-round")
        res = {m: [] for m in modes}
        for m in modes:
            step(mode=m)
            step(mode=m)
        for _trial in range(2):
            for m in modes:
                step(mode=m)
                dist.barrier()
                torch.cuda.synchronize()
                tp = time.perf_counter()
                for _ in range(5):
                    step(mode=m)
                torch.cuda.synchronize()
                dist.barrier()
                t = torch.tensor([time.perf_counter() - tp], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                res[m].append(float(t.item()) / 5 * 1e3)
        best = {m: min(v) for m, v in res.items()}
        one_launch = best["one"] <= best["per-round"]
        _lib.call("fa_step_record", skey.encode(), 1 if one_launch else 0)  # for the product and later runs
        mode_probe = {"one_launch_ms": round(best["one"], 4), "per_round_ms": round(best["per-round"], 4),
                      "chosen": "one launch" if one_launch else "per round",
                      "how": "wall time of 5 steps between barriers, max over ranks, best of 2 trials per form",
                      "recorded": skey}
    elif can_one and recorded >= 0:
        mode_probe = {"chosen": "one launch" if one_launch else "per round", "restored": skey,
                      "how": "recorded by an earlier probe (fa_step_lookup): no timing run"}
    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    warm_extra = 0
    if args.warmup_s > 0:
        spent = time.perf_counter() - tw
        per = spent / max(1, args.warmup)
        warm_extra = max(0, min(10_000, int((args.warmup_s - spent) / max(per, 1e-6)) + 1)) if spent < args.warmup_s \
            else 0
        if dist_on:  # every rank runs the same number of steps (each has collectives)
            t = torch.tensor([warm_extra], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            warm_extra = int(t.item())
        for _ in range(warm_extra):
            step()
    if product and agg.one_launch == "probe" and rounds > 1:
        # the class's probe alternates the forms over its first PROBE_STEPS
        # calls of the shape; the timed steps run the form it keeps (the same
        # count of calls on every rank: its decision is max-over-ranks timing)
        for _ in range(agg.PROBE_STEPS):
            if agg.step_form(wl.X, lay) is not None:
                break
            step()
            warm_extra += 1
        pkey = agg.step_key(wl.X, lay)
        got = agg.probed.get(pkey)
        mode_probe = ({"chosen": agg.step_form(wl.X, lay), "recorded": pkey,
                       "one_launch_ms": [round(x, 4) for x in got["one"]],
                       "per_round_ms": [round(x, 4) for x in got["per"]],
                       "how": "ShardedAggregator(one_launch='probe'): its first PROBE_STEPS calls alternate "
                              "the forms, PROBE_WARM untimed calls of each, then PROBE_CALLS timed back to back "
                              "(device time per call, max over ranks); the best call of each compared"}
                      if got else {"chosen": agg.step_form(wl.X, lay), "restored": pkey,
                                   "how": "recorded in the tuner's cache file (fa_step_lookup), rank 0's record "
                                          "broadcast: no timing run"})
    evs = [([(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
             for _ in range(rounds)], torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if product:
        agg.trace = []  # the class records its own fold / end events per call
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    # One GPU: the folds run back to back and two events bracket the whole timed
    # region (per-launch events would add their own few-microsecond gaps to
    # every launch, which distorts the small models).  Several GPUs: events
    # around every round's fold split a step into fold time and exposed gather.
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    region[0].record(stream)
    for k in range(args.steps):
        step(evs[k] if dist_on else None)
    if product and args.check == "deferred":
        agg.check_timeouts()  # the pipelined caller's check, inside the timed region
    region[1].record(stream)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if product:
        evs, agg.trace = agg.trace, None
        # the form the timed calls ran: one fold launch per call, or one per round
        one_launch = rounds > 1 and all(len(folds) == 1 for folds, _ in evs)
        # this rank's own slots folded by the per-round product launches: the
        # gather check's and the CPU baseline's reference for the product's model
        for k in range(rounds):
            wl.launch(0, k)
        torch.cuda.synchronize()
    gather_ok = None
    if px is not None:
        # the whole model the peer copy reassembled must equal an RCCL step's, bit for bit
        peer_full = full.clone()
        full.zero_()
        step_one_launch(exchange="rccl")
        torch.cuda.synchronize()
        t = torch.tensor([1 if torch.equal(peer_full.view(torch.uint8), full.view(torch.uint8)) else 0],
                         dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        gather_ok = bool(t.item())
        del peer_full
    elif dist_on:
        # the whole reassembled model: my slots in my copy are my fold output,
        # bit for bit, and every rank's copy is the same model (two position-
        # weighted digests of its bits agree on all ranks), so every rank's
        # slots are right in every copy
        ok = True
        iv = torch.int32 if wl.dtype == "f32" else torch.int16
        for k, (lo, hi) in enumerate(wl.slots):
            if hi > lo:
                ok &= torch.equal(full[lo:hi].view(iv), send[lay.offset(k):lay.offset(k) + hi - lo].view(iv))
        dig = model_digest(full.view(iv))
        t = torch.cat([torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev), dig, -dig])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)  # own-slot flags; digests' min and -max
        gather_ok = bool(t[0].item() == 1 and torch.equal(t[1:3], -t[3:5]))
    if dist_on and one_launch:
        # one fold launch per step: its span (events around it), and the
        # exchange left exposed after it (from the launch's end to the step's)
        kern_ms = [folds[0][0].elapsed_time(folds[0][1]) for folds, _ in evs]
        exposed_ms = [folds[0][1].elapsed_time(end) for folds, end in evs]
        kern_avg = float(np.mean(kern_ms))
        exposed_avg = float(np.mean(exposed_ms))
        round_ms = [float(np.median(kern_ms))]
    elif dist_on:
        kern_ms = [sum(e0.elapsed_time(e1) for e0, e1 in folds) for folds, _ in evs]
        # the exchange left exposed: from the last fold's end to the end of the step
        exposed_ms = [folds[-1][1].elapsed_time(end) for folds, end in evs]
        kern_avg = float(np.mean(kern_ms))
        exposed_avg = float(np.mean(exposed_ms))
        # each round's fold (median over the steps): beside the previous round's
        # all-gather from round 1 on, alone in round 0 (RCCL's kernels share the CUs)
        round_ms = [float(np.median([folds[k][0].elapsed_time(folds[k][1]) for folds, _ in evs]))
                    for k in range(rounds)]
    else:
        kern_avg = region[0].elapsed_time(region[1]) / args.steps  # per fold call, launch gaps included
        exposed_avg = 0.0
        round_ms = None
    timeouts = None
    if dist_on:
        t = torch.tensor([kern_avg, exposed_avg, *round_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        kern_avg, exposed_avg = float(t[0].item()), float(t[1].item())
        round_ms = [round(float(x), 4) for x in t[2:].tolist()]
    if can_one:  # a round wait that gave up (never expected) let an exchange read an unfinished round
        fstream = sharding_fold_stream(dev) if product else stream  # where the step's fold launches ran
        n_to = max(0, L.fa_rounds_timeouts(engine.rounds_state(dev, fstream.cuda_stream)))
        for p in ([px] if px is not None else []) + ([q for q in agg._peers.values() if q is not None]
                                                     if product else []):
            n_to += max(0, L.fa_rounds_timeouts(p.state)) + max(0, L.fa_rounds_check(p.state))
        t = torch.tensor([n_to], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        timeouts = int(t.item())

    # streaming-read ceiling over the same HBM bytes (contiguous, no fold)
    # byte-level sweep: bf16 input is read as the same bytes viewed as fp32 quads
    nfl = wl.N * wl.P * wl.X.element_size() // 4
    sink = torch.empty(8192, dtype=torch.float32, device=dev)
    ts = []
    for k in range(max(3, min(args.steps, 10)) + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        _lib.check(B.fa_read_sweep_f32(wl.X.data_ptr(), nfl - nfl % 4, sink.data_ptr(), 8192,
                                       stream.cuda_stream), "read_sweep", bench=True)
        e1.record(stream)
        e1.synchronize()
        if k >= 2:
            ts.append(e0.elapsed_time(e1))
    ceiling = (nfl - nfl % 4) * 4 / (sorted(ts)[len(ts) // 2] * 1e-3) / 1e9

    tb = torch.tensor([float(wl.bytes)], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(tb)  # units all ranks processed
    total_bytes = float(tb.item()) * args.steps
    value = total_bytes / elapsed / 1e9
    achieved = wl.bytes / (kern_avg * 1e-3) / 1e9
    # the committed PMC pass measured exactly this launch: the unmodified config, one fold per step
    traffic, traffic_src = (read_traffic(args.config) if not (args.clients or args.params) and rounds == 1
                            else (None, None))
    if traffic is not None and wl.dtype == "f32" and args.variant == 0:
        # the committed pass measured the policy's form; another measured choice is another kernel
        form = L.fa_fold_form(1, wl.N, lay.width(0), wl.ldx, 1 if wl.scored else 0, stream.cuda_stream).decode()
        pol = B.fa_f32_pick_name(wl.N, lay.width(0), 0).decode()
        if form != pol:
            traffic, traffic_src = None, f"{traffic_src}: measured form {pol}, this run took {form}"
    devices = rank_devices(dev)
    cpu = None
    # the CPU baseline runs on rank 0 at every world size, after the timed
    # region (the other ranks wait at the barrier below), so every line -- the
    # N-GPU ones included -- carries the reference timed on the same host
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(wl, args.cpu_cols, args.cpu_reps)
        except Exception as e:  # the baseline must never hide the GPU result
            cpu = {"error": repr(e)}
        if world == 1 and not args.no_full_lean:
            try:
                cpu["full_lean"] = cpu_full_lean(wl)
            except Exception as e:
                cpu["full_lean"] = {"error": repr(e)}
    if dist_on:
        dist.barrier()
    if rank == 0:
        line = {
            "metric": "aggregated GB/s (device-resident) — N-client FedAvg fp32 reduction",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_extra_steps": warm_extra,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": wl.scaling,
            "vs_baseline": None,
            "dtype": "f32" if wl.dtype == "f32" else "bf16-in/f32-acc",
            "data": "synthetic (integer-exact splitmix64 generator, generated in HBM)",
            "config": {
                "workload": wl.desc,
                "clients": wl.N,
                "params_per_gpu": wl.P,
                "params_total": wl.P_total,
                "layout": f"row-stacked [clients][params] {'fp32' if wl.dtype == 'f32' else 'bf16'} in HBM",
                "row_pitch": wl.ldx,
                "parallelism": f"param-bucket x{world}" + (
                    f" + {'RCCL' if backend == 'nccl' else backend} all_gather in {rounds} rounds overlapped with "
                    "the fold" if dist_on else ""),
                "rounds": rounds,
                "round_widths": lay.widths,
                "fold_stream": "high priority" if dist_on else "default",
                "fold_launch": ("one launch per step (fa_fedavg_*_rounds), each round's all-gather behind its "
                                "completion flag" if one_launch else
                                "one launch per round" if dist_on else "one launch"),
                "fold_form_by_rank_own_choice": forms_by_rank,
                "fold_form_ranks_agreed": forms_agree,
                "fold_form_rank0_broadcast": bool(dist_on and world > 1 and args.variant == 0 and per_round_possible),
                "step_mode": step_mode if dist_on and rounds > 1 else None,
                "step_impl": ("product: ShardedAggregator(one_launch=%r, exchange=%r, check=%r).aggregate_slots per "
                              "step" % (agg.one_launch, agg.exchange, agg.check)) if product else
                             ("loop (bench.py's own step)" if dist_on else None),
                "outputs": ("fp32" if wl.dtype == "f32" else
                            "RNE bf16 only (the exchanged form; no fp32 result, ABI 5)" if not wl.write_f32 else
                            "fp32 + RNE bf16"),
                "exchange": (args.exchange if one_launch else "rccl") if dist_on else None,
                "step_mode_probe": mode_probe,
                "variant": "splitn (opt-in, not bit-exact)" if args.variant < 0 else
                (B.fa_variant_name if wl.dtype == "f32" else B.fa_bf16_variant_name)(args.variant).decode(),
                # the kernel form the product's fp32 auto fold takes for one launch of this rank
                # the kernel form each distinct slot width ran (the tuner's measured choice), and the
                # shape policy's form for the first slot (what runs with FEDAVG_AUTOTUNE=0)
                "fold_form": (L.fa_rounds_form(1 if wl.dtype == "bf16" else 0).decode() if one_launch else
                              {str(w): L.fa_fold_form(1 if wl.dtype == "f32" else 2, wl.N, w, wl.ldx,
                                                      1 if wl.scored else 0, stream.cuda_stream).decode()
                               for w in dict.fromkeys(lay.widths)} if args.variant == 0 else None),
                "fold_policy": (B.fa_f32_pick_name(wl.N, lay.sub, 0).decode()
                                if wl.dtype == "f32" and args.variant == 0 and not args.unpadded else None),
                "autotune": {"on": bool(L.fa_set_autotune(-1)), "tuning_calls": tune_calls,
                             "pending": L.fa_autotune_pending()},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_ms_avg": round(kern_avg, 4),
                "read_sweep_ceiling": round(ceiling, 1),
                "frac_of_read_ceiling": round(achieved / ceiling, 4),
                "bytes_per_launch": wl.bytes,
            },
            "cpu_baseline": cpu,
            "gather_check": gather_ok,
            # the ranks that actually ran: torch.distributed's world and each rank's GPU
            "dist": {"backend": backend, "world_size": dist.get_world_size() if dist_on else 1,
                     "launcher": ("in-process one-rank group (--rccl-world1)" if args.rccl_world1 else
                                  "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ or
                                  "GROUP_RANK" in os.environ else
                                  "environment (WORLD_SIZE set)" if dist_on else "none (single process)"),
                     "devices": devices},
            # per-rank split of a step at N > 1 (max over ranks): the fold kernels,
            # and the all-gather left exposed after the last fold of the step
            "fold_ms": round(kern_avg, 4),
            "fold_ms_per_round": round_ms if not one_launch else None,
            "fold_ms_per_step_launch_median": round_ms[0] if one_launch else None,
            "round_wait_timeouts": timeouts,
            "gather_exposed_ms": round(exposed_avg, 4) if dist_on else None,
            "gather_bytes_per_rank": (lay.padded_total * (4 if wl.dtype == "f32" else 2)
                                      * (world - 1) // world) if dist_on else 0,
        }
        print(json.dumps(line), file=out, flush=True)
        if timeouts:
            # an exchange behind a timed-out round wait read an unfinished round: the
            # line above is reported, the run fails (ShardedAggregator raises the same)
            from fedlesscan_amd.aggregator.exceptions import AggregationError
            raise AggregationError(f"{timeouts} round wait(s) timed out during the run")
    if px is not None:
        px.close()
    if agg is not None:
        agg.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
