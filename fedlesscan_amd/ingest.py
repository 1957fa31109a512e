"""Pipelined host ingest: client rows -> pinned staging -> H2D -> in-order fold.

The reference materialises every decoded client (aggregation.py:87-93) and
then folds on one CPU core.  Here client rows are packed, in arrival order,
into pinned host chunks of `chunk_rows` rows; each full chunk is copied to the
GPU on a dedicated copy stream while the previous chunk is folded on the
compute stream with fa_fold_f32 (accumulator carried across chunks, divide
once at the end).  Folding in chunks with a carried accumulator performs the
same additions in the same order, so the result is bit-identical to one
fa_fedavg_f32 over all rows (tests/test_gpu_parity.py checks this).

With direct=True, rows whose layers already sit in page-locked memory (a
pinned result store, fedlesscan_amd.pinned) skip the packing copy: each layer
is DMA'd from where it lies straight into its row of the device chunk
(fa_copy_h2d on the copy stream), as soon as the row is added.  Other rows are
packed with fa_pack and copied in runs of consecutive packed rows.  It is off
by default: on MI355X hosts the 16-thread pack fully overlaps the DMA, and one
copy per chunk beat one copy per layer; it pays where host memcpy
bandwidth, not PCIe, is the limit.

Memory: `slots` pinned + `slots` device chunks of chunk_rows x P floats (2 by
default; FEDAVG_STREAM_SLOTS overrides) and one [P] accumulator, independent of
the number of clients.  More, smaller chunks shorten the exposed tail of a
round (the last chunk's DMA and fold run after the last row arrives) at the
cost of more copies and launches.
"""
from __future__ import annotations

import collections
import ctypes
import os
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .aggregator.exceptions import InvalidParameterShapeError
from .engine import round_scalars


class StreamingFold:
    """Accumulate fp32 client rows on the GPU in order; `finish()` divides.

    add(row, weight, score=None): row = flat float32 [P] (or a list of layers
    that flatten to P), weight = the client's cardinality (Python scalar, rounded
    to fp32 like numpy), score = stall-aware factor or None.  Either every row
    has a score or none does.
    """

    # process-wide row counts by ingest route (diagnostics; tests check the route)
    stats = {"direct_rows": 0, "packed_rows": 0}

    def __init__(self, P: int, chunk_rows: int = 16, device: Optional[torch.device] = None,
                 pitch_align: int = 64, direct: bool = False, slots: Optional[int] = None):
        if P <= 0:
            raise InvalidParameterShapeError("StreamingFold needs P > 0")
        self.P = P
        self.dev = device or torch.device("cuda", torch.cuda.current_device())
        self.ldx = ((P + pitch_align - 1) // pitch_align) * pitch_align
        self.R = max(1, chunk_rows)
        K = self.K = max(2, slots if slots is not None else int(os.environ.get("FEDAVG_STREAM_SLOTS", "2")))
        self.host = [torch.empty((self.R, self.ldx), dtype=torch.float32, pin_memory=True) for _ in range(K)]
        # per-chunk factors [a; s] travel with the chunk's rows on the copy
        # stream, from pinned memory (a pageable H2D could stall the producer)
        self.fac_host = [torch.empty((2, self.R), dtype=torch.float32, pin_memory=True) for _ in range(K)]
        self.fac_dev = [torch.empty((2, self.R), dtype=torch.float32, device=self.dev) for _ in range(K)]
        self.devbuf = [torch.empty((self.R, self.ldx), dtype=torch.float32, device=self.dev) for _ in range(K)]
        self.acc = torch.empty(P, dtype=torch.float32, device=self.dev)
        self.copy_stream = torch.cuda.Stream(device=self.dev)
        self.compute = torch.cuda.current_stream(self.dev)
        self.h2d_done = [torch.cuda.Event() for _ in range(K)]
        self.fold_done = [torch.cuda.Event() for _ in range(K)]
        self.fold_pending = [False] * K
        self.buf = 0
        self.fill = 0
        self.weights: List = []
        self.scored: Optional[bool] = None
        self.chunk_a: List = [[] for _ in range(K)]
        self.chunk_s: List = [[] for _ in range(K)]
        self.started = False
        self.rows = 0
        # per chunk: source layers and their byte offsets inside the pinned chunk
        self.srcs: List = [[] for _ in range(K)]
        # per chunk: which rows were DMA'd directly, and the arrays those copies read
        self.row_direct: List = [[] for _ in range(K)]
        self.keep: List = [[] for _ in range(K)]
        self.direct = direct
        self.direct_rows = 0
        self.threads = int(os.environ.get("FEDAVG_COPY_THREADS", "0")) or min(16, os.cpu_count() or 1)

    # -- producer side ------------------------------------------------------
    def _slot_ready(self, b: int):
        # the pinned buffer b may be overwritten once its last H2D finished;
        # its device twin once the fold that read it finished
        if self.fold_pending[b]:
            self.fold_done[b].synchronize()
            self.fold_pending[b] = False
        self.keep[b] = []  # their direct copies finished before that fold ran

    def add(self, row, weight, score: Optional[float] = None):
        if self.scored is None:
            self.scored = score is not None
        elif self.scored != (score is not None):
            raise InvalidParameterShapeError("either every row has a score or none does")
        b = self.buf
        if self.fill == 0:
            self._slot_ready(b)
        pieces = row if isinstance(row, (list, tuple)) else [row]
        base = self.fill * self.ldx * 4
        total = 0
        arrs = []
        for layer in pieces:
            arr = np.ascontiguousarray(layer)
            if arr.dtype != np.float32:
                raise InvalidParameterShapeError(f"StreamingFold takes float32 rows, got {arr.dtype}")
            arrs.append((arr, base + 4 * total))
            total += arr.size
        if total != self.P:
            raise InvalidParameterShapeError(f"row has {total} parameters, expected {self.P}")
        L = _lib.load()
        if self.direct and all(L.fa_host_is_pinned(a.ctypes.data, a.nbytes) for a, _ in arrs if a.nbytes):
            dst = self.devbuf[b].data_ptr()
            cs = self.copy_stream.cuda_stream
            for a, off in arrs:
                _lib.check(L.fa_copy_h2d(dst + off, a.ctypes.data, a.nbytes, cs), "fa_copy_h2d")
            self.keep[b].extend(a for a, _ in arrs)
            self.row_direct[b].append(True)
            self.direct_rows += 1
            StreamingFold.stats["direct_rows"] += 1
        else:
            self.srcs[b].extend(arrs)
            self.row_direct[b].append(False)
            StreamingFold.stats["packed_rows"] += 1
        self.weights.append(weight)
        self.chunk_a[b].append(weight)
        self.chunk_s[b].append(score)
        self.fill += 1
        self.rows += 1
        if self.fill == self.R:
            self._flush()

    def _pack(self, b: int):
        """Copy the chunk's layers into pinned buffer b with fa_pack (C++ threads, GIL released)."""
        entries = self.srcs[b]
        if not entries:
            return
        n = len(entries)
        offs = np.fromiter((o for _, o in entries), dtype=np.int64, count=n)
        ptrs = np.fromiter((a.ctypes.data for a, _ in entries), dtype=np.uint64, count=n)
        sizes = np.fromiter((a.nbytes for a, _ in entries), dtype=np.int64, count=n)
        _lib.call("fa_pack", self.host[b].data_ptr(), offs.ctypes.data, ptrs.ctypes.data, sizes.ctypes.data, n,
                  self.threads)
        self.srcs[b] = []

    def _flush(self, finalize: bool = False, total=None):
        b, n = self.buf, self.fill
        self._pack(b)  # every row of this chunk is in pinned memory before its H2D
        if n:
            with torch.cuda.stream(self.copy_stream):
                direct = self.row_direct[b]
                r = 0
                while r < n:  # runs of packed rows; direct rows are already on their way
                    if direct[r]:
                        r += 1
                        continue
                    r1 = r + 1
                    while r1 < n and not direct[r1]:
                        r1 += 1
                    self.devbuf[b][r:r1].copy_(self.host[b][r:r1], non_blocking=True)
                    r = r1
                fh = self.fac_host[b].numpy()
                fh[0, :n] = round_scalars(self.chunk_a[b], np.float32)  # fl32(n_i), numpy's rounding
                scored = self.chunk_s[b][0] is not None
                if scored:
                    fh[1, :n] = round_scalars(self.chunk_s[b], np.float32)
                self.fac_dev[b].copy_(self.fac_host[b], non_blocking=True)
                self.h2d_done[b].record(self.copy_stream)
            self.compute.wait_event(self.h2d_done[b])
            a = self.fac_dev[b][0]
            s = self.fac_dev[b][1] if scored else None
        div = float(np.float32(sum(self.weights) if total is None else total)) if finalize else 0.0
        L = _lib.load()
        st = self.compute.cuda_stream
        if n:
            _lib.check(L.fa_fold_f32(self.devbuf[b].data_ptr(), n, self.P, self.ldx, a.data_ptr(),
                                     None if s is None else s.data_ptr(),
                                     self.acc.data_ptr() if self.started else None, div, int(finalize),
                                     self.acc.data_ptr(), st), "fa_fold_f32")
            self.started = True
            self.fold_done[b].record(self.compute)
            self.fold_pending[b] = True
        elif finalize:
            _lib.check(L.fa_fold_f32(None, 0, self.P, self.ldx, None, None, self.acc.data_ptr(), div, 1,
                                     self.acc.data_ptr(), st), "fa_fold_f32(finalize)")
        self.chunk_a[b], self.chunk_s[b] = [], []
        self.row_direct[b] = []
        self.fill = 0
        self.buf = (self.buf + 1) % self.K

    def finish(self, total=None) -> torch.Tensor:
        """Fold the last partial chunk and divide by fl32(total or sum(weights))."""
        if self.rows == 0:
            _lib.check(_lib.FA_ERR_NO_CLIENTS, "StreamingFold.finish")
        self._flush(finalize=True, total=total)
        if any(self.keep):
            # direct copies read the callers' arrays: they must be done before
            # the caller may free them
            self.copy_stream.synchronize()
            self.keep = [[] for _ in range(self.K)]
        return self.acc

    def abandon(self):
        """Give up this round (a caller falling back to another path): wait for
        the copies already issued, drop the row references."""
        self.copy_stream.synchronize()
        self.keep = [[] for _ in range(self.K)]


class _PipeCache:
    """Native ingest pipes (fa_ingest_*) kept across rounds: a pipe owns
    page-locked and device chunks and an issuer thread, so it is created once
    per (device, P, chunk size, slots) and reused; a pipe serves one round at a
    time (a concurrent round gets its own), and at most MAX idle pipes are
    kept per process."""

    MAX = 4

    def __init__(self):
        self.lock = threading.Lock()
        self.idle: "collections.OrderedDict" = collections.OrderedDict()  # key -> [pipe, ...]

    def get(self, key):
        with self.lock:
            pipes = self.idle.get(key)
            if pipes:
                p = pipes.pop()
                if not pipes:
                    del self.idle[key]
                return p
        dev, P, chunk_bytes, slots = key
        h = ctypes.c_void_p()
        _lib.call("fa_ingest_create", ctypes.byref(h), P, chunk_bytes, slots, dev)
        return h

    def put(self, key, pipe):
        with self.lock:
            self.idle.setdefault(key, []).append(pipe)
            self.idle.move_to_end(key)
            n = sum(len(v) for v in self.idle.values())
            while n > self.MAX:
                k, v = next(iter(self.idle.items()))
                _lib.load().fa_ingest_destroy(v.pop())
                if not v:
                    del self.idle[k]
                n -= 1

    @staticmethod
    def drop(pipe):
        _lib.load().fa_ingest_destroy(pipe)


_pipes = _PipeCache()


class NativeStreamingFold:
    """StreamingFold on the native pipe (libfedavg_hip.so fa_ingest_*): the
    same add(row, weight, score) / finish(total) contract and bit-identical
    result, with the packing done by the library's copy workers and the DMA and
    fold issued by its own thread, so add() returns as soon as the row's copies
    are queued and decoding the next row overlaps everything else.  The rows'
    arrays are kept alive until finish() (the workers read them)."""

    stats = {"rows": 0}

    def __init__(self, P: int, device: Optional[torch.device] = None, chunk_bytes: int = 16 << 20,
                 slots: int = 4, expected_rows: int = 0):
        if P <= 0:
            raise InvalidParameterShapeError("StreamingFold needs P > 0")
        self.P = P
        self.dev = device or torch.device("cuda", torch.cuda.current_device())
        if self.dev.index is None:
            self.dev = torch.device("cuda", torch.cuda.current_device())
        self.key = (self.dev.index, P, int(chunk_bytes), int(slots))
        self.pipe = _pipes.get(self.key)
        self.acc = torch.empty(P, dtype=torch.float32, device=self.dev)
        self.L = _lib.load()
        try:
            _lib.check(self.L.fa_ingest_begin(self.pipe, self.acc.data_ptr(),
                                              torch.cuda.current_stream(self.dev).cuda_stream,
                                              max(0, int(expected_rows))), "fa_ingest_begin")
        except BaseException:
            _pipes.drop(self.pipe)
            self.pipe = None
            raise
        self.keep: List = []
        self.weights: List = []
        self.rows = 0

    def _fail(self):
        if self.pipe is not None:  # a round that failed half-way is not reused
            _pipes.drop(self.pipe)
            self.pipe = None
        self.keep = []

    def add(self, row, weight, score: Optional[float] = None):
        if self.pipe is None:
            raise InvalidParameterShapeError("this StreamingFold failed earlier")
        pieces = row if isinstance(row, (list, tuple)) else [row]
        arrs = []
        for layer in pieces:
            arr = np.ascontiguousarray(layer)
            if arr.dtype != np.float32:
                self._fail()
                raise InvalidParameterShapeError(f"StreamingFold takes float32 rows, got {arr.dtype}")
            arrs.append(arr)
        n = len(arrs)
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
        sizes = (ctypes.c_int64 * n)(*[a.nbytes for a in arrs])
        a = float(np.float32(weight))  # fl32(n_i): numpy's rounding of the Python scalar
        s = 1.0 if score is None else float(np.float32(score))
        rc = self.L.fa_ingest_add(self.pipe, ptrs, sizes, n, a, s, 0 if score is None else 1)
        if rc:
            err = _lib.last_error()
            self._fail()
            if rc == _lib.FA_ERR_SHAPE:
                raise InvalidParameterShapeError(f"fa_ingest_add: {err}")
            _lib.check(rc, "fa_ingest_add")
        self.keep.append(arrs)
        self.weights.append(weight)
        self.rows += 1
        NativeStreamingFold.stats["rows"] += 1

    def finish(self, total=None) -> torch.Tensor:
        if self.pipe is None:
            raise InvalidParameterShapeError("this StreamingFold failed earlier")
        if self.rows == 0:
            self._fail()
            _lib.check(_lib.FA_ERR_NO_CLIENTS, "StreamingFold.finish")
        div = float(np.float32(sum(self.weights) if total is None else total))
        rc = self.L.fa_ingest_finish(self.pipe, div)
        if rc:
            err = _lib.last_error()
            self._fail()
            _lib.check(rc, f"fa_ingest_finish ({err})")
        _pipes.put(self.key, self.pipe)  # every copy is done: the rows are no longer read
        self.pipe = None
        self.keep = []
        return self.acc

    def abandon(self):
        """Give up this round now (a caller that falls back to another path):
        the pipe is destroyed here -- its copies waited for, its issuer thread
        joined -- rather than left issuing for an accumulator nobody reads until
        garbage collection runs __del__."""
        if self.pipe is not None:
            _pipes.drop(self.pipe)
            self.pipe = None
        self.keep = []

    def __del__(self):
        if getattr(self, "pipe", None) is not None:  # abandoned mid-round
            try:
                _pipes.drop(self.pipe)
            except Exception:
                pass


# native pipe by default; FEDAVG_NATIVE_INGEST=0 selects the Python-driven StreamingFold
NATIVE_INGEST = os.environ.get("FEDAVG_NATIVE_INGEST", "1") == "1"
STREAM_SLOTS = int(os.environ.get("FEDAVG_STREAM_SLOTS", "0"))  # 0: the form's default


def chunk_class(nbytes: int, cap: int) -> int:
    """The chunk size a pipe is made (and cached) for: the next power of two
    >= nbytes, at least 1 MiB, at most cap.  A round whose rows need less than
    a full chunk rounds up to a few size classes, so rounds whose client count
    varies (stragglers, failures) reuse the same pipe instead of each creating
    and destroying its own page-locked slots and issuer thread."""
    c = 1 << 20
    while c < nbytes and c < cap:
        c <<= 1
    return min(c, cap)


def make_streaming_fold(P: int, device, chunk_bytes: int, direct: bool = False, expected_rows: int = 0):
    """The ingest for P-float rows on `device`: the native pipe, or the
    Python-driven StreamingFold for the direct-DMA route (page-locked
    documents) or when FEDAVG_NATIVE_INGEST=0.  expected_rows: the round's row
    count when the caller knows it (the native pipe then shrinks its last
    chunks)."""
    if NATIVE_INGEST and not direct:
        return NativeStreamingFold(P, device, chunk_bytes, STREAM_SLOTS or 3, expected_rows)
    return StreamingFold(P, chunk_rows=max(1, chunk_bytes // (4 * P)), device=device, direct=direct,
                         slots=STREAM_SLOTS or None)


def stream_layers(rows_iter, shapes: Sequence[tuple], chunk_rows: int = 16, device=None):
    """Convenience: fold an iterator of (layers, weight[, score]) tuples."""
    P = sum(int(np.prod(s)) if len(s) else 1 for s in shapes)
    sf = StreamingFold(P, chunk_rows=chunk_rows, device=device)
    for item in rows_iter:
        layers, w = item[0], item[1]
        sc = item[2] if len(item) > 2 else None
        sf.add(layers, w, sc)
    return sf.finish()
