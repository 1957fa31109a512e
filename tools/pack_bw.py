#!/usr/bin/env python3
"""Host pack bandwidth on the GPU box (diagnostics): fa_pack of 400 MB of
pageable rows into page-locked staging, alone and with the DMA engine reading
other page-locked memory at the same time (the ingest pipe's steady state).
Run once with FEDAVG_PACK_NT=1 (streaming stores, default) and once with 0."""
import ctypes
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


def main():
    L = _lib.load()
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
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pack()
        ts.append(time.perf_counter() - t0)
    res["pack_alone_gbs"] = round(n_rows * row * 4 / min(ts) / 1e9, 1)
    # with a concurrent H2D stream of other pinned memory
    dev = torch.device("cuda", 0)
    h = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
    d = torch.empty_like(h, device=dev)
    stop = threading.Event()

    def dma():
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            while not stop.is_set():
                d.copy_(h, non_blocking=True)
                s.synchronize()

    th = threading.Thread(target=dma)
    th.start()
    time.sleep(0.2)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pack()
        ts.append(time.perf_counter() - t0)
    stop.set()
    th.join()
    res["pack_with_dma_gbs"] = round(n_rows * row * 4 / min(ts) / 1e9, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
