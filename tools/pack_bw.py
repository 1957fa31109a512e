#!/usr/bin/env python3
"""Host pack bandwidth on the GPU box (diagnostics).

Default: fa_pack of 400 MB of pageable rows into page-locked staging, alone
and with the DMA engine reading other page-locked memory at the same time
(the ingest pipe's steady state).  Run once with FEDAVG_PACK_NT=1 (streaming
stores, default) and once with 0.

--buckets 1,2,4,8 (round 5): the single-process multi-GPU
drop-in (multigpu.MultiStreamingFold, aggregation.py:95-97 ->
fed_avg_aggregator.py:67-69) hands every decoded client row to G ingest pipes,
one per GPU, each packing its own column bucket of the row into its own
page-locked chunks.  This packs G buckets at once from NPZ-decoded rows (the
zero-copy views npz.native_views gives of real NPZ blobs, as
serialization.py:280-306 decodes them) into G page-locked regions, one
fa_pack over every bucket's pieces of every row split by bytes over 16 x G
threads (`--threads-per-bucket` x G: the ingest pipes' shared copy pool grows
by 16 workers per GPU, ingest_pipe.cpp CopyPool).  Reports the aggregate GB/s
per G, alone and beside a concurrent H2D stream, against the G x pinned-H2D
rate the G GPUs' PCIe links would take.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from fedlesscan_amd import _lib  # noqa: E402


def single(L):
    n_rows, row = 100, 1_000_000
    src = [np.random.default_rng(i).standard_normal(row).astype(np.float32) for i in range(n_rows)]
    dst = torch.empty(n_rows * row, dtype=torch.float32, pin_memory=True)
    offs = np.arange(n_rows, dtype=np.int64) * row * 4
    ptrs = np.array([a.ctypes.data for a in src], dtype=np.uint64)
    sizes = np.full(n_rows, row * 4, dtype=np.int64)
    threads = int(os.environ.get("FEDAVG_COPY_THREADS", "16"))

    def pack():
        _lib.check(L.fa_pack(dst.data_ptr(), offs.ctypes.data, ptrs.ctypes.data, sizes.ctypes.data, n_rows, threads),
                   "fa_pack")

    pack()
    res = {"nt": os.environ.get("FEDAVG_PACK_NT", "1"), "threads": threads}
    res["pack_alone_gbs"] = round(n_rows * row * 4 / best_of(pack, 5) / 1e9, 1)
    with DmaLoad():
        res["pack_with_dma_gbs"] = round(n_rows * row * 4 / best_of(pack, 5) / 1e9, 1)
    print(json.dumps(res), flush=True)


def best_of(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


class DmaLoad:
    """A background H2D stream of page-locked memory (the copy engine's reads
    of host memory while the workers pack); .gbs = its rate meanwhile."""

    def __enter__(self):
        dev = torch.device("cuda", 0)
        self.h = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
        self.d = torch.empty_like(self.h, device=dev)
        self.stop = threading.Event()
        self.moved = 0

        def dma():
            s = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                while not self.stop.is_set():
                    self.d.copy_(self.h, non_blocking=True)
                    s.synchronize()
                    self.moved += self.h.numel()

        self.th = threading.Thread(target=dma)
        self.t0 = time.perf_counter()
        self.th.start()
        time.sleep(0.2)
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()
        self.gbs = self.moved / (time.perf_counter() - self.t0) / 1e9


def h2d_rate():
    dev = torch.device("cuda", 0)
    h = torch.empty(512 << 20, dtype=torch.uint8, pin_memory=True)
    d = torch.empty_like(h, device=dev)
    d.copy_(h)
    torch.cuda.synchronize()

    def once():
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
    return h.numel() / best_of(once, 5) / 1e9


def buckets(L, args):
    from fedlesscan_amd import npz
    from fedlesscan_amd.multigpu import _bucket_pieces, _layer_offsets, column_buckets
    N, P = args.rows, args.params
    # a model of four layers (a dense layer the size of most of the model), as the
    # C3 end-to-end blobs (bench_e2e.py): every client's blob written by write_npz
    sizes = [P // 2, P // 4, P // 8, P - P // 2 - P // 4 - P // 8]
    rng = np.random.default_rng(7)
    base = [rng.standard_normal(s).astype(np.float32) for s in sizes]
    blobs = []
    for i in range(N):
        blobs.append(npz.write_npz([b + np.float32(i) for b in base]))
    rows = [npz.native_views(b) for b in blobs]  # zero-copy views into the blobs
    assert all(r is not None for r in rows)
    rate = h2d_rate()
    out = {"rows": N, "params": P, "row_bytes": P * 4, "threads_per_bucket": args.threads_per_bucket,
           "pinned_h2d_gbs_one_link": round(rate, 1), "host_cpus": os.cpu_count(), "by_buckets": []}
    flats = [[x.reshape(-1) for x in layers] for layers in rows]
    loffs = _layer_offsets(flats[0])
    dst = torch.empty(N * P + 64 * 16, dtype=torch.float32, pin_memory=True)
    for G in [int(g) for g in args.buckets.split(",") if g]:
        ptrs, szs, offs = [], [], []
        region = 0  # bucket g's rows side by side at its own region of dst (as its pipe's chunks)
        for (lo, hi) in column_buckets(P, G):
            w = hi - lo
            if w <= 0:
                continue
            for i in range(N):
                o = (region + i * w) * 4
                for p in _bucket_pieces(flats[i], loffs, lo, hi):
                    ptrs.append(p.ctypes.data)
                    szs.append(p.nbytes)
                    offs.append(o)
                    o += p.nbytes
            region += N * w
        offs, ptrs, szs = np.array(offs, np.int64), np.array(ptrs, np.uint64), np.array(szs, np.int64)
        T = G * args.threads_per_bucket

        def pack_all():
            _lib.check(L.fa_pack(dst.data_ptr(), offs.ctypes.data, ptrs.ctypes.data, szs.ctypes.data, len(szs), T),
                       "fa_pack")

        pack_all()
        total = N * P * 4
        alone = total / best_of(pack_all, args.reps) / 1e9
        with DmaLoad() as dma:
            beside = total / best_of(pack_all, args.reps) / 1e9
        need = G * rate
        rec = {"G": G, "workers": T, "pieces": int(len(szs)), "pack_gbs": round(alone, 1),
               "pack_gbs_beside_h2d": round(beside, 1), "h2d_during_gbs": round(dma.gbs, 1),
               "links_need_gbs": round(need, 1), "ceiling_gbs": round(min(beside, need), 1),
               "bound": "pack" if beside < need else "pcie"}
        out["by_buckets"].append(rec)
        print(json.dumps(rec), flush=True)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", default="", help="comma-separated bucket counts G (multi-GPU drop-in packing)")
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--threads-per-bucket", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    L = _lib.load()
    if args.buckets:
        buckets(L, args)
    else:
        single(L)


if __name__ == "__main__":
    main()
