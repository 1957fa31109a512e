#!/usr/bin/env python3
"""Time bf16 fold forms (fa_bf16_form_name) on one shape with the inputs in
HBM: each form 3 untimed + `--reps` timed launches between events, two
interleaved passes, and every form's outputs compared bit for bit with the
first one's.

    python tools/bf16_forms_bench.py --clients 256 --params 100000000 --forms bf16_bands2_u2c8,bf16_bands2_u4c8
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=256)
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--forms", required=True)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = _lib.load_bench()
    names = {B.fa_bf16_form_name(i).decode(): i for i in range(B.fa_num_bf16_forms())}
    forms = [f for f in args.forms.split(",") if f]
    N, P = args.clients, args.params
    ldx = (P + 63) // 64 * 64
    st = torch.cuda.current_stream(dev)
    X = torch.empty((N, ldx), dtype=torch.bfloat16, device=dev)
    _lib.check(B.fa_synth_bf16(X.data_ptr(), N, P, ldx, 5, 0, 0, st.cuda_stream), "synth", bench=True)
    w = synth.cardinalities(5, N)
    a = torch.tensor(np.array(w, np.float32), device=dev)
    div = float(np.float32(sum(w)))
    out = {f: (torch.empty(P, dtype=torch.float32, device=dev), torch.empty(P, dtype=torch.int16, device=dev))
           for f in forms}
    gb = (N * P * 2 + P * 6) / 1e9

    def run(f):
        o, ob = out[f]
        _lib.check(B.fa_fedavg_bf16_form(X.data_ptr(), N, P, ldx, a.data_ptr(), None, div, o.data_ptr(),
                                         ob.data_ptr(), st.cuda_stream, names[f]), f, bench=True)

    times = {f: [] for f in forms}
    for f in forms:
        for _ in range(3):
            run(f)
    torch.cuda.synchronize()
    for _pass in range(2):
        for f in forms:
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                run(f)
                e1.record(st)
                e1.synchronize()
                times[f].append(e0.elapsed_time(e1))
    ref = forms[0]
    for f in forms:
        t = sorted(times[f])
        same = torch.equal(out[f][0].view(torch.int32), out[ref][0].view(torch.int32)) and \
            torch.equal(out[f][1], out[ref][1])
        print(f"{f:24s} median {t[len(t) // 2]:.4f} ms  min {t[0]:.4f} ms  {gb / (t[len(t) // 2] * 1e-3):8.1f} GB/s"
              f"  same bits as {ref}: {same}", flush=True)


if __name__ == "__main__":
    main()
