#!/usr/bin/env python3
"""Host-side cost of one engine.fold_stacked call, piece by piece (GPU box).

    python tools/host_overhead.py [--clients N] [--params P]  -> one JSON line

Host microseconds per call (median of perf_counter spans around the call,
the GPU drained before each one), for the whole call and for its parts:
factor rounding, factor staging (pinned ring + async H2D), the output
allocation, the stream query and the ctypes launch.  For a small model the GPU
waits for this work between back-to-back calls.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import _lib, engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--clients", type=int, default=1024)
ap.add_argument("--params", type=int, default=67267)
ap.add_argument("--reps", type=int, default=500)
args = ap.parse_args()
dev = torch.device("cuda", 0)
N, P = args.clients, args.params
X = torch.empty((N, P), dtype=torch.float32, device=dev)
_lib.check(_lib.load_bench().fa_synth_f32(X.data_ptr(), N, P, P, 9, 0, 0, engine.stream_ptr(dev)), "synth",
           bench=True)
w = synth.cardinalities(9, N)
sc = [(r + 1) / 11 for r in synth.round_ids(9, N, 10, 2)]
torch.cuda.synchronize()


def us(fn):
    """Median host time of one call (perf_counter around the call), the GPU
    drained before each call so the call never waits for earlier work (the
    factor slots of the library, the caching allocator)."""
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 2)


f = engine.Factors(w, None, np.dtype(np.float32))
rows = [X[i].clone() for i in range(N)]
rs = engine.RowSet(rows)
rs_views = engine.RowSet([X[i] for i in range(N)])
wl = list(w)
res = {
    "clients": N, "params": P,
    "fold_stacked_us": us(lambda: engine.fold_stacked(X, w)),
    "fold_stacked_scored_us": us(lambda: engine.fold_stacked(X, w, sc)),
    "result_dtype_us": us(lambda: engine.result_dtype(np.dtype(np.float32), w, None)),
    "factors_us": us(lambda: engine.Factors(w, None, np.dtype(np.float32))),
    "factors_scored_us": us(lambda: engine.Factors(w, sc, np.dtype(np.float32))),
    "stage_us": us(lambda: f.to(dev)),
    "empty_out_us": us(lambda: torch.empty(P, dtype=torch.float32, device=dev)),
    "stream_ptr_us": us(lambda: engine.stream_ptr(dev)),
    "fold_rows_rowset_us": us(lambda: engine.fold_rows(rs, w)),
    "fold_rows_views_rowset_us": us(lambda: engine.fold_rows(rs_views, w)),
    "sum_weights_us": us(lambda: sum(wl)),
    "round_scalars_us": us(lambda: engine.round_scalars(wl, np.dtype(np.float32))),
    "type_set_us": us(lambda: set(map(type, wl))),
}
a, _ = f.to(dev)
out = torch.empty(P, dtype=torch.float32, device=dev)
st = engine.stream_ptr(dev)
L = _lib.load()
ah = f.a
res["hostf_launch_us"] = us(lambda: L.fa_fedavg_f32_hostf(X.data_ptr(), N, P, P, ah.ctypes.data, None, float(f.div),
                                                         out.data_ptr(), st))
res["ctypes_launch_us"] = us(lambda: L.fa_fedavg_f32(X.data_ptr(), N, P, P, a.data_ptr(), None, float(f.div),
                                                     out.data_ptr(), st))
print(json.dumps(res))
