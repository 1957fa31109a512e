#!/usr/bin/env python3
"""What the tuner measures (FEDAVG_AUTOTUNE_LOG=1 prints each decision with
every candidate's best time): one shape, tuned with the calls isolated (a
device synchronize after each, as the bench's tuning pass and one aggregation
round per FL round) or back to back (--b2b: no synchronize until the end).
The first call's wall time is also given in folds of the chosen form: with a
warm cache file (--cache PATH, written by an earlier process) a known shape's
first call is one fold.  --vary-clients N1,N2,...: one call per client count
(the straggler-driven rounds of FL), each call's wall time.

    FEDAVG_AUTOTUNE_LOG=1 python tools/tuner_probe.py --clients 100 --params 300000 [--b2b] [--cache PATH]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--params", type=int, default=300000)
    ap.add_argument("--b2b", action="store_true")
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--cache", default=None, help="tuner cache file (FEDAVG_TUNE_CACHE); '0' = off")
    ap.add_argument("--vary-clients", default="", help="comma-separated client counts, one call each")
    args = ap.parse_args()
    if args.cache is not None:
        os.environ["FEDAVG_TUNE_CACHE"] = args.cache
    N, P = max([args.clients] + [int(x) for x in args.vary_clients.split(",") if x]), args.params
    dev = torch.device("cuda", 0)
    L, B = _lib.load(), _lib.load_bench()
    st = torch.cuda.current_stream(dev).cuda_stream
    ldx = (P + 63) // 64 * 64
    X = torch.empty((N, ldx), dtype=torch.bfloat16 if args.bf16 else torch.float32, device=dev)
    gen = B.fa_synth_bf16 if args.bf16 else B.fa_synth_f32
    _lib.check(gen(X.data_ptr(), N, P, ldx, 7, 0, 0, st), "synth", bench=True)
    a = torch.tensor(np.array(synth.cardinalities(7, N), np.float32), device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    div = float(a.sum().item())
    kind = 2 if args.bf16 else 1

    def call(n=None):
        n = N if n is None else n
        if args.bf16:
            _lib.check(L.fa_fedavg_bf16(X.data_ptr(), n, P, ldx, a.data_ptr(), None, div, out.data_ptr(), None, st),
                       "bf16")
        else:
            _lib.check(L.fa_fedavg_f32(X.data_ptr(), n, P, ldx, a.data_ptr(), None, div, out.data_ptr(), st), "f32")

    if args.vary_clients:
        for n in [int(x) for x in args.vary_clients.split(",") if x]:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            call(n)
            torch.cuda.synchronize()
            print(f"vary {n}x{P}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
        return

    # load the library's code object first (a fold of an unrelated small shape),
    # so the first call below pays the tuner's cost, not the process's first launch
    tiny = torch.zeros((3, 1024), dtype=X.dtype, device=dev)
    tout = torch.empty(1024, dtype=torch.float32, device=dev)
    if args.bf16:
        _lib.check(L.fa_fedavg_bf16(tiny.data_ptr(), 3, 1024, 1024, a.data_ptr(), None, 1.0, tout.data_ptr(), None, st),
                   "warm-up")
    else:
        _lib.check(L.fa_fedavg_f32(tiny.data_ptr(), 3, 1024, 1024, a.data_ptr(), None, 1.0, tout.data_ptr(), st),
                   "warm-up")
    # the first call of the shape (it runs every candidate form), wall time to completion
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call()
    torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    n = 0
    for n in range(1, 400):
        call()
        if not args.b2b:
            torch.cuda.synchronize()
        if n % 8 == 0 or not args.b2b:
            if args.b2b:
                torch.cuda.synchronize()
            if L.fa_fold_form(kind, N, P, ldx, 0, st):
                break
    form = L.fa_fold_form(kind, N, P, ldx, 0, st).decode()
    # the chosen form, timed back to back
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        call()
    e1.record()
    e1.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call()
    torch.cuda.synchronize()
    later_ms = (time.perf_counter() - t0) * 1e3
    fold_ms = e0.elapsed_time(e1) / 50
    print(f"{'b2b' if args.b2b else 'isolated'} {N}x{P}: first call {first_ms:.2f} ms "
          f"(= {first_ms / fold_ms:.1f} folds of the chosen form), a later call {later_ms:.3f} ms, then {n} calls -> "
          f"{form}, back-to-back {fold_ms:.4f} ms; cache {L.fa_tune_export(None, 0)} bytes of decisions, file "
          f"{os.environ.get('FEDAVG_TUNE_CACHE', 'default')}", flush=True)


if __name__ == "__main__":
    main()
