#!/usr/bin/env python3
"""End-to-end aggregation rate from host-resident serialized client blobs.

    python bench_e2e.py [--clients N] [--params P] [--reps R] [--bson [--pinned-store]]

What the reference's aggregator function actually does per round
(aggregation.py:87-97, fed_avg_aggregator.py:57-92): N ClientResult objects
holding NPZ blobs -> decode -> weighted fold -> parameters.  Timed here:

  gpu_e2e   FedAvgAggregator.aggregate(ClientResults) of this package: zero-copy
            NPZ views -> pinned chunks -> H2D (copy stream) -> in-order chunked
            HIP fold -> D2H of the result, returned as numpy layers
  cpu_ref   the oracle's restatement of the same call (np.load decode + numpy
            fold on one core), i.e. the reference's own cost on this host
  h2d       pinned host->device copy bandwidth of the same bytes (PCIe bound)

With --bson the results start where the reference keeps them: one BSON
document per client in the (in-memory) result store, as GridFS holds them
(client_daos.py:73).  gpu_e2e then includes the store read and the native BSON
walk (blob stays a view); cpu_ref includes pymongo's bson.decode (the
reference's own codec, client_daos.py:142) before the np.load + numpy fold.
--pinned-store keeps those documents in page-locked memory and turns on the
direct route: the ingest DMAs every layer straight from its document, with no
packing copy (engine.DIRECT_DMA).

Rates are input bytes (N * P * 4) per second.  Results are compared bit for bit.
Writes one JSON line (rank 0, one GPU).  Not the headline metric: DESIGN.md.
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from fedlesscan_amd import FedAvgAggregator, synth  # noqa: E402
from fedlesscan_amd.common.models import (ClientResult, NpzWeightsSerializerConfig,  # noqa: E402
                                          SerializedParameters, WeightsSerializerConfig)

MNIST_LIKE = [(5, 5, 1, 32), (32,), (5, 5, 32, 64), (64,), (1024, 512), (512,), (512, 10), (10,)]


def make_blobs(N, P, seed):
    from oracle import oracle_lib as OL  # fast host generator (test/bench infrastructure)
    from fedlesscan_amd.npz import write_npz  # byte-identical to np.savez, threaded CRC
    blobs = []
    for i in range(N):
        row = OL.synth_f32(seed, 1, P, row0=i)[0]
        # split the row into a few layers like a Keras get_weights() list
        cuts = [0, P // 64, P // 8, P // 2, P]
        layers = [row[cuts[k]:cuts[k + 1]].reshape(-1, 1) if k % 2 else row[cuts[k]:cuts[k + 1]]
                  for k in range(4)]
        blob = write_npz(layers)
        if blob is None:
            f = io.BytesIO()
            np.savez(f, *layers)
            blob = f.getvalue()
        blobs.append(blob)
    return blobs


def check_columns(out, N, P, seed, cards, ncols):
    """GPU result vs the C oracle (the reference op order, fed_avg_aggregator.py:31-41)
    on the first and the last `ncols` columns, regenerated on the host."""
    from oracle import oracle_lib as OL
    flat = np.concatenate([np.asarray(x).reshape(-1) for x in out])
    a = np.array(cards, np.float32)
    div = np.float32(sum(cards))
    ok = True
    for c0 in sorted({0, max(0, P - ncols)}):
        nc = min(ncols, P - c0)
        exp = OL.fedavg_f32(OL.synth_f32(seed, N, nc, col0=c0), a, div)
        ok &= bool(np.array_equal(flat[c0:c0 + nc].view(np.uint32), exp.view(np.uint32)))
    return ok


def results(blobs, cards):
    cfg = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())
    return [ClientResult(parameters=SerializedParameters(blob=b, serializer=cfg), cardinality=c)
            for b, c in zip(blobs, cards)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--params", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check-cols", type=int, default=0,
                    help="with --no-cpu: check the first and last K output columns against the C oracle")
    ap.add_argument("--bson", action="store_true", help="start from BSON documents in the result store")
    ap.add_argument("--pinned-store", action="store_true", help="with --bson: documents in page-locked memory")
    ap.add_argument("--devices", default="",
                    help="comma-separated GPU ordinals for the multi-GPU drop-in (FedAvgAggregator(devices=...)); "
                         "'all' = every visible GPU; a GPU may repeat (buckets sharing one GPU)")
    a = ap.parse_args()
    from oracle import fedavg_oracle as O  # checker + CPU reference timing only
    N, P = a.clients, a.params
    t0 = time.time()
    blobs = make_blobs(N, P, a.seed)
    cards = synth.cardinalities(a.seed, N)
    gen_s = time.time() - t0
    in_bytes = N * P * 4
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    store = None
    if a.pinned_store:
        from fedlesscan_amd import engine
        engine.DIRECT_DMA = True
    if a.bson or a.pinned_store:
        from fedlesscan_amd.store import InMemoryClientResultStore
        store = InMemoryClientResultStore(pinned=a.pinned_store)
        for i, cr in enumerate(results(blobs, cards)):
            store.save("bench", 1, f"client-{i}", cr)

    devices = None
    if a.devices:
        devices = "all" if a.devices == "all" else [int(x) for x in a.devices.split(",")]

    def one_round(crs):
        if store is not None:
            agg = FedAvgAggregator(devices=devices)
            feats, it = agg.select_aggregation_candidates(store, "bench", 1)
            return agg.aggregate(list(it), feats)
        return FedAvgAggregator(devices=devices).aggregate(crs, None)

    # warm up the pipeline (pinned allocations, library load)
    FedAvgAggregator(devices=devices).aggregate(results(blobs[: min(N, 4)], cards[: min(N, 4)]), None)
    torch.cuda.synchronize()
    ts, out = [], None
    for _ in range(a.reps):
        crs = None if store is not None else results(blobs, cards)
        t0 = time.perf_counter()
        out, _ = one_round(crs)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t_gpu = sorted(ts)[len(ts) // 2]
    from fedlesscan_amd.ingest import NATIVE_INGEST, NativeStreamingFold, StreamingFold
    routes = dict(StreamingFold.stats)
    routes["native_pipe_rows"] = NativeStreamingFold.stats["rows"]

    # decode-only (zero-copy views) and pinned H2D of the same bytes
    from fedlesscan_amd.npz import read_layers
    t0 = time.perf_counter()
    for b in blobs:
        read_layers(b)
    t_decode = time.perf_counter() - t0
    host = torch.empty(min(in_bytes // 4, 1 << 28), dtype=torch.float32, pin_memory=True)
    dbuf = torch.empty_like(host, device=dev)
    dbuf.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dbuf.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbs = 3 * host.numel() * 4 / (time.perf_counter() - t0) / 1e9

    res = {
        "metric": "end-to-end aggregation GB/s from host NPZ blobs (not the headline)",
        "source": ("BSON documents in a page-locked result store" if a.pinned_store else
                   "BSON documents in the result store" if a.bson else "ClientResult objects holding NPZ blobs"),
        "clients": N, "params": P, "input_bytes": in_bytes, "gen_s": round(gen_s, 1),
        "gpu_e2e_s": round(t_gpu, 4), "gpu_e2e_gbs": round(in_bytes / t_gpu / 1e9, 2),
        "gpu_e2e_min_s": round(min(ts), 4), "gpu_e2e_max_s": round(max(ts), 4),
        "stream_chunk_mb": int(os.environ.get("FEDAVG_STREAM_CHUNK_MB", "32")),
        "stream_slots": int(os.environ.get("FEDAVG_STREAM_SLOTS", "0")) or None,
        "ingest": "native pipe (fa_ingest_*)" if NATIVE_INGEST and not a.pinned_store else "python StreamingFold",
        "decode_views_s": round(t_decode, 4), "h2d_pinned_gbs": round(h2d_gbs, 1),
        "ingest_rows": routes,
        "devices": a.devices or "current GPU",
    }
    if a.no_cpu and a.check_cols > 0:
        t0 = time.perf_counter()
        res["bit_exact_column_sample"] = check_columns(out, N, P, a.seed, cards, a.check_cols)
        res["column_sample"] = f"first and last {min(a.check_cols, P)} columns vs the C oracle"
        res["check_s"] = round(time.perf_counter() - t0, 1)
    if not a.no_cpu:
        if store is not None:
            import bson  # pymongo's codec: the reference's own decode (CPU leg only)
            files = [store._files[d["file_id"]] for d in store._docs]
            files = [f if isinstance(f, bytes) else bytes(f) for f in files]  # untimed: GridFS hands bytes
        t0 = time.perf_counter()
        if store is not None:
            docs = [bson.decode(f) for f in files]
            dicts = [{"blob": d["parameters"]["blob"], "cardinality": d["cardinality"]} for d in docs]
        else:
            dicts = [{"blob": b, "cardinality": c} for b, c in zip(blobs, cards)]
        ref, _ = O.aggregate_fedavg(dicts)
        t_cpu = time.perf_counter() - t0
        res["cpu_ref_s"] = round(t_cpu, 3)
        res["cpu_ref_gbs"] = round(in_bytes / t_cpu / 1e9, 3)
        res["cpu_ref_cores"] = 1
        res["speedup_vs_cpu_ref"] = round(t_cpu / t_gpu, 1)
        res["bit_exact"] = all(np.array_equal(x.view(np.uint32), y.view(np.uint32)) and x.shape == y.shape
                               for x, y in zip(out, ref))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
