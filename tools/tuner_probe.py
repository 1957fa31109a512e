#!/usr/bin/env python3
"""What the tuner measures (FEDAVG_AUTOTUNE_LOG=1 prints each decision with
every candidate's best time): one shape, tuned with the calls isolated (a
device synchronize after each, as the bench's tuning pass and one aggregation
round per FL round) or back to back (--b2b: no synchronize until the end).

    FEDAVG_AUTOTUNE_LOG=1 python tools/tuner_probe.py --clients 100 --params 300000 [--b2b]
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
    args = ap.parse_args()
    N, P = args.clients, args.params
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

    def call():
        if args.bf16:
            _lib.check(L.fa_fedavg_bf16(X.data_ptr(), N, P, ldx, a.data_ptr(), None, div, out.data_ptr(), None, st),
                       "bf16")
        else:
            _lib.check(L.fa_fedavg_f32(X.data_ptr(), N, P, ldx, a.data_ptr(), None, div, out.data_ptr(), st), "f32")

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
    print(f"{'b2b' if args.b2b else 'isolated'} {N}x{P}: first call {first_ms:.2f} ms (measures every form), "
          f"a later call {later_ms:.3f} ms, then {n} calls -> {form}, back-to-back {e0.elapsed_time(e1) / 50:.4f} ms",
          flush=True)


if __name__ == "__main__":
    main()
