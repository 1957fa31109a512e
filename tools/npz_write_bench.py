#!/usr/bin/env python3
"""Saving the aggregated model: np.savez (the reference's NpzWeightsSerializer)
against fedlesscan_amd.npz.write_npz (byte-identical, native checksums), on the
model shapes of the BASELINE configs.  Host only; one JSON line per model.

    python tools/npz_write_bench.py [--reps 5]
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd.npz import write_npz  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
models = {
    # mnist/model.py:4-23, 582,026 params
    "C1 MNIST CNN (8 layers)": [(5, 5, 1, 32), (32,), (5, 5, 32, 64), (64,), (1024, 512), (512,), (512, 10), (10,)],
    "C2 1M params": [(1_000_000,)],
    "C3 10M params": [(10_000_000,)],
    "C4 100M params fp32": [(100_000_000,)],
}
rng = np.random.default_rng(0)
for name, shapes in models.items():
    arrs = [rng.standard_normal(s).astype(np.float32) for s in shapes]

    def savez():
        f = io.BytesIO()
        np.savez(f, *arrs)
        return f.getvalue()

    def med(fn):
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return sorted(ts)[len(ts) // 2]

    same = write_npz(arrs) == savez()
    t_ref, t_new = med(savez), med(lambda: write_npz(arrs))
    nbytes = sum(a.nbytes for a in arrs)
    print(json.dumps({"model": name, "bytes": nbytes, "np_savez_ms": round(t_ref * 1e3, 2),
                      "write_npz_ms": round(t_new * 1e3, 2), "speedup": round(t_ref / t_new, 2),
                      "write_npz_GBps": round(nbytes / t_new / 1e9, 2), "byte_identical": same,
                      "threads": os.environ.get("OMP_NUM_THREADS")}))
