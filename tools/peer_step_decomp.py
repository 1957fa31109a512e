#!/usr/bin/env python3
"""Where the world-1 peer-copy step's time goes.

One 8-GPU C4 rank's step on the one GPU (256 clients x overlap_layout(100M,
8, "bf16"), or --config c3: 1024 x a C3 rank's fp32 slots), no process group:
each line is K back-to-back calls between two events on the fold stream, the
median of --reps interleaved repetitions.

  fold_agent       the policy one-launch fold, rounds published at agent scope
                   (a bench-library rounds state, sys 0: sc1 tile stores)
  fold_sys         the same at system scope as a peer exchange's state (sys 1:
                   sc0 sc1 tile stores, no per-block fence, the product)
  fold_sys_fence   round 5's system publication (sys 2: sc1 stores and a
                   system release fence per block and round)
  self_copy        hipMemcpyAsync of the step's exchanged bytes, device to
                   device on one GPU (the world-1 peer step's only copy)
  peer_step        PeerExchange.step: fence, the fold (sys 1), per round a
                   flag wait and the copy on a copy stream, the ack
  product_peer     ShardedAggregator(one_launch=True, exchange="peer_copy")
                   .aggregate_slots, check="deferred" (one check at the end)
  product_rccl     ShardedAggregator(one_launch=True) at world 1 (the rounds'
                   self-copies behind their waits), check="deferred"
  product_sync     product_rccl with check="sync" (a host wait per call)
  product_per      ShardedAggregator(one_launch=False): per-round launches
  *_traced         product_rccl / product_per with .trace on (bench.py's timing
                   events around every fold launch, the cost they add)
  *_dflt           product_rccl / product_per called from the default stream
                   (the class hops onto the fold stream and back: the hops' cost)

The same command under `rocprofv3 --kernel-trace --memory-copy-trace` names
the engine that moves each copy (a blit kernel in the kernel trace, or an
SDMA entry in the copy trace) and the hardware queue of every dispatch.

    python tools/peer_step_decomp.py [--config c4|c3] [--steps 20] [--reps 5] [--only a,b]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import _lib, synth  # noqa: E402
from fedlesscan_amd.engine import Factors  # noqa: E402
from fedlesscan_amd.sharding import PeerExchange, ShardedAggregator, fold_stream, gather_stream, overlap_layout  # noqa


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=["c4", "c3"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="comma-separated line names")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    L, B = _lib.load(), _lib.load_bench()
    if args.config == "c4":
        N, P_total, world, dt = 256, 100_000_000, 8, "bf16"
    else:
        N, P_total, world, dt = 1024, 80_000_000, 8, "f32"
    bf16 = dt == "bf16"
    # one rank's share as a world-1 layout (the same round shares: widths within
    # an alignment unit of the 8-rank layout's per-rank slots)
    lay = overlap_layout(P_total // world, 1, dt)
    W = lay.local_width
    st0 = torch.cuda.current_stream(dev)
    X = torch.empty((N, W), dtype=torch.bfloat16 if bf16 else torch.float32, device=dev)
    gen = B.fa_synth_bf16 if bf16 else B.fa_synth_f32
    _lib.check(gen(X.data_ptr(), N, W, W, 21, 0, 0, st0.cuda_stream), "synth", bench=True)
    w = synth.cardinalities(21, N)
    a, _ = Factors(w, None, np.dtype(np.float32)).to(dev)
    div = float(np.float32(sum(w)))
    odt = torch.bfloat16 if bf16 else torch.float32
    send = torch.empty(W, dtype=odt, device=dev)
    dst = torch.empty(W, dtype=odt, device=dev)
    offs = (ctypes.c_int64 * (lay.rounds + 1))(*[lay.offset(k) for k in range(lay.rounds + 1)])
    fs, gs = fold_stream(dev), gather_stream(dev)
    pol = L.fa_rounds_form(1 if bf16 else 0).decode()
    form = next(i for i in range(B.fa_num_step_forms()) if B.fa_step_form_name(i).decode() == pol)
    states = {}
    for sysm in (0, 1, 2):
        h = ctypes.c_void_p()
        _lib.check(B.fa_bench_rounds_create(ctypes.byref(h), 0), "rounds", bench=True)
        _lib.check(B.fa_bench_rounds_set_sys(h, sysm), "sys", bench=True)
        states[sysm] = h
    nbytes = N * lay.P * (2 if bf16 else 4) + lay.P * (2 if bf16 else 4)

    def fold(sysm):
        o, ob = (None, send.data_ptr()) if bf16 else (send.data_ptr(), None)
        _lib.check(B.fa_fedavg_rounds_form(states[sysm], form, X.data_ptr(), N, W, a.data_ptr(), None, div, o, ob,
                                           lay.rounds, offs, fs.cuda_stream), "fold", bench=True)

    px = PeerExchange(None, dev, lay, bf16)
    full = torch.empty(lay.padded_total, dtype=odt, device=dev)
    aggs = {"product_peer": ShardedAggregator(one_launch=True, exchange="peer_copy", check="deferred"),
            "product_rccl": ShardedAggregator(one_launch=True, check="deferred"),
            "product_sync": ShardedAggregator(one_launch=True, check="sync"),
            "product_per": ShardedAggregator(one_launch=False, check="deferred")}
    for n in ("product_rccl", "product_per"):
        for sfx in ("_traced", "_dflt"):
            aggs[n + sfx] = ShardedAggregator(one_launch=n == "product_rccl", check="deferred")
            if sfx == "_traced":
                aggs[n + sfx].trace = []

    def run(name):
        if name in ("fold_agent", "fold_sys", "fold_sys_fence"):
            fold({"fold_agent": 0, "fold_sys": 1, "fold_sys_fence": 2}[name])
        elif name == "self_copy":  # the copy on the fold stream, alone
            with torch.cuda.stream(fs):
                dst.copy_(send)
        elif name == "peer_step":
            px.step(X, w, None, full, None, fs, gs)
            fs.wait_stream(gs)
        elif name.endswith("_dflt"):
            aggs[name].aggregate_slots(X, w, None, lay, out=full)
        else:
            with torch.cuda.stream(fs):
                aggs[name].aggregate_slots(X, w, None, lay, out=full)

    names = ["fold_agent", "fold_sys", "fold_sys_fence", "self_copy", "peer_step", "product_peer", "product_rccl",
             "product_sync", "product_per", "product_rccl_traced", "product_per_traced", "product_rccl_dflt",
             "product_per_dflt"]
    if args.only:
        names = [n for n in names if n in args.only.split(",")]
    for n in names:  # warm-up (first launches, the tuner's per-round shapes, buffers)
        for _ in range(3):
            run(n)
    torch.cuda.synchronize()
    res = {n: [] for n in names}
    rng = np.random.default_rng(7)
    for _ in range(args.reps):
        order = list(names)
        rng.shuffle(order)
        for n in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(fs)
            for _ in range(args.steps):
                run(n)
            if n.startswith("product") and aggs[n].check == "deferred":
                aggs[n].check_timeouts()
            fs.wait_stream(torch.cuda.current_stream(dev))
            e1.record(fs)
            e1.synchronize()
            res[n].append(e0.elapsed_time(e1) / args.steps)
            if n.endswith("_traced"):
                aggs[n].trace.clear()
    # every product / peer model equals the agent-scope fold's output, bit for bit
    fold(0)
    torch.cuda.synchronize()
    ref = send.clone()
    px.step(X, w, None, full, None, fs, gs)
    fs.wait_stream(gs)
    torch.cuda.synchronize()
    P = lay.P
    exact = {"peer_step": bool(torch.equal(full[:P].view(torch.uint8), ref[:P].view(torch.uint8)))}
    for n, agg in aggs.items():
        got = agg.aggregate_slots(X, w, None, lay)
        torch.cuda.synchronize()
        exact[n] = bool(torch.equal(got.view(torch.uint8), ref[:P].view(torch.uint8)))
        if agg.check == "deferred":
            agg.check_timeouts()
    timeouts = max(0, L.fa_rounds_timeouts(px.state))
    med = {n: float(np.median(v)) for n, v in res.items()}
    out = {"config": args.config, "clients": N, "slot_widths": lay.widths, "params": lay.P, "dtype": dt,
           "step_form": pol, "bytes_per_step": nbytes, "steps_per_rep": args.steps, "reps": args.reps,
           "ms_median": {n: round(v, 4) for n, v in med.items()},
           "ms_all": {n: [round(x, 4) for x in v] for n, v in res.items()},
           "gbs": {n: round(nbytes / (v * 1e-3) / 1e9, 1) for n, v in med.items() if not n.startswith("self")},
           "vs_fold_agent": ({n: round(v / med["fold_agent"], 4) for n, v in med.items()}
                             if "fold_agent" in med else None),
           "bit_exact_vs_fold": exact, "peer_wait_timeouts": timeouts}
    print(json.dumps(out), flush=True)
    for agg in aggs.values():
        agg.close()
    px.close()


if __name__ == "__main__":
    main()
