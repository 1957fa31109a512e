#!/usr/bin/env python3
"""Phase breakdown of one end-to-end aggregation round (GPU; diagnostics only).

    python tools/e2e_phases.py [--clients N] [--params P] [--pinned-store]

Times, with a device synchronize at every boundary: store read + BSON/NPZ
decode, StreamingFold setup, the add() loop (host issue), finish(), the wait for
the device, the D2H of the result.  Also: the same bytes as 1 big and as N
row-sized pinned H2D copies, to separate DMA limits from pipeline overheads.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--pinned-store", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    sys.path.insert(0, REPO)
    import bench_e2e as BE
    from fedlesscan_amd import FedAvgAggregator, synth
    from fedlesscan_amd.aggregator.fed_avg_aggregator import decode_results
    from fedlesscan_amd.engine import STREAM_CHUNK_BYTES
    from fedlesscan_amd.ingest import make_streaming_fold
    from fedlesscan_amd.store import InMemoryClientResultStore
    from fedlesscan_amd.engine import to_host as engine_to_host
    N, P = a.clients, a.params
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    blobs = BE.make_blobs(N, P, 2)
    cards = synth.cardinalities(2, N)
    store = InMemoryClientResultStore(pinned=a.pinned_store)
    for i, cr in enumerate(BE.results(blobs, cards)):
        store.save("s", 1, f"c{i}", cr)
    FedAvgAggregator().aggregate(BE.results(blobs[:2], cards[:2]), None)
    torch.cuda.synchronize()
    out = []
    for rep in range(a.reps):
        t = [time.perf_counter()]
        feats, it = FedAvgAggregator().select_aggregation_candidates(store, "s", 1)
        params, w, _ = decode_results(list(it), None)
        t.append(time.perf_counter())
        rows = max(1, min(N, STREAM_CHUNK_BYTES // (4 * P)))
        sf = make_streaming_fold(P, dev, STREAM_CHUNK_BYTES)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        for i in range(N):
            sf.add(params[i], w[i])
        t.append(time.perf_counter())
        acc = sf.finish()
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        engine_to_host(acc)
        t.append(time.perf_counter())
        names = ["decode", "setup", "adds", "finish", "device_wait", "d2h"]
        out.append({k: round((t[j + 1] - t[j]) * 1e3, 2) for j, k in enumerate(names)})
        out[-1]["total"] = round((t[-1] - t[0]) * 1e3, 2)
    # raw DMA: one big copy vs N row copies from pinned memory
    host = torch.empty(N * P, dtype=torch.float32, pin_memory=True)
    d = torch.empty_like(host, device=dev)
    d.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    one = time.perf_counter() - t0
    hv, dv = host.view(N, P), d.view(N, P)
    t0 = time.perf_counter()
    for i in range(N):
        dv[i].copy_(hv[i], non_blocking=True)
    torch.cuda.synchronize()
    rows_t = time.perf_counter() - t0
    print(json.dumps({"clients": N, "params": P, "pinned_store": a.pinned_store, "chunk_rows": rows,
                      "phases_ms": out, "dma_one_copy_ms": round(one * 1e3, 2),
                      "dma_row_copies_ms": round(rows_t * 1e3, 2),
                      "dma_gbs": round(N * P * 4 / one / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
