"""Single-process multi-GPU aggregation: one column bucket per GPU.

The reference calls the aggregation strategy in-process, once per round
(aggregation.py:71-97 -> FedAvgAggregator.aggregate, fed_avg_aggregator.py:
57-92).  `sharding.py` scales the fold with one process per GPU under
torch.distributed; this module scales the drop-in itself: the same strategy
object, called the same way, folds on several GPUs of the node.

Every output column is independent (one lane owns a column and
adds the clients in order), so the model's P columns are cut into one
contiguous, 64-element-aligned bucket per GPU (sharding.bucket_bounds) and each
GPU folds ALL clients of its bucket with the same HIP kernels.  Nothing is
reduced across GPUs: the result is bit-identical to the one-GPU fold by
construction, for any number of GPUs.

  MultiStreamingFold   host rows (decoded NPZ blobs, the input of aggregate())
                       -> each GPU packs, DMAs and folds only its own columns:
                       one PCIe link per GPU carries 1/G of the bytes, so the
                       end-to-end rate is not capped by one link
  fold_stacked_multi   device-resident buckets [N, P_g] on their GPUs -> the
                       [P] model on one GPU, reassembled with fa_copy_peer
                       (hipMemcpyPeerAsync over xGMI)
  scatter_columns      host [N, P] -> per-GPU buckets (test and simulation helper)

The same device may appear several times in `devices` (e.g. the one GPU of a
test box): each entry then gets its own bucket and streams on that GPU.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .aggregator.exceptions import InvalidParameterShapeError
from .sharding import bucket_bounds


def resolve_devices(devices) -> List[torch.device]:
    """A list of CUDA (HIP) devices from ints, strings or torch.device objects;
    "all" = every visible GPU."""
    if isinstance(devices, str) and devices == "all":
        devices = list(range(torch.cuda.device_count()))
    if isinstance(devices, (int, str, torch.device)):
        devices = [devices]
    out = []
    for d in devices:
        dev = torch.device("cuda", d) if isinstance(d, int) else torch.device(d)
        if dev.type != "cuda":
            raise ValueError(f"multi-GPU aggregation needs CUDA (HIP) devices, got {dev}")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        out.append(dev)
    if not out:
        raise ValueError("no devices given")
    return out


def column_buckets(P: int, n_devices: int) -> List[tuple]:
    """[lo, hi) of every GPU's columns: equal 64-element-aligned buckets, the
    last one short (possibly empty for tiny models)."""
    return bucket_bounds(P, n_devices)


def _layer_offsets(layers) -> np.ndarray:
    sizes = [int(np.prod(np.shape(x))) if np.ndim(x) else 1 for x in layers]
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)


def _bucket_pieces(flat: List[np.ndarray], offs: np.ndarray, lo: int, hi: int) -> List[np.ndarray]:
    """Zero-copy views of the flattened layers covering columns [lo, hi)."""
    pieces = []
    for li in range(len(flat)):
        a, b = max(lo, int(offs[li])), min(hi, int(offs[li + 1]))
        if a < b:
            pieces.append(flat[li][a - offs[li]:b - offs[li]])
    return pieces


class MultiStreamingFold:
    """StreamingFold (ingest.py) over several GPUs, one column bucket each.

    add(layers, weight, score=None) takes one client's layers (float32 numpy
    arrays flattening to P, in the reference's client order); each GPU receives
    only its columns of the row (zero-copy views of the layers, packed into
    that GPU's pinned chunks).  finish() divides on every GPU and returns the
    [P] model in page-locked host memory, each bucket copied D2H on its own GPU.
    """

    def __init__(self, P: int, devices: Sequence, chunk_bytes: int = 64 << 20, direct: bool = False,
                 expected_rows: int = 0):
        from .ingest import make_streaming_fold
        if P <= 0:
            raise InvalidParameterShapeError("MultiStreamingFold needs P > 0")
        self.P = P
        self.devices = resolve_devices(devices)
        self.bounds = column_buckets(P, len(self.devices))
        self.folds = []
        for dev, (lo, hi) in zip(self.devices, self.bounds):
            w = hi - lo
            self.folds.append(make_streaming_fold(w, dev, chunk_bytes, direct=direct, expected_rows=expected_rows)
                              if w > 0 else None)
        self.rows = 0

    def add(self, layers, weight, score: Optional[float] = None):
        layers = layers if isinstance(layers, (list, tuple)) else [layers]
        flat = []
        for x in layers:
            arr = np.ascontiguousarray(x)
            if arr.dtype != np.float32:
                raise InvalidParameterShapeError(f"MultiStreamingFold takes float32 rows, got {arr.dtype}")
            flat.append(arr.reshape(-1))
        offs = _layer_offsets(flat)
        if int(offs[-1]) != self.P:
            raise InvalidParameterShapeError(f"row has {int(offs[-1])} parameters, expected {self.P}")
        for sf, (lo, hi) in zip(self.folds, self.bounds):
            if sf is not None:
                sf.add(_bucket_pieces(flat, offs, lo, hi), weight, score)
        self.rows += 1

    def abandon(self):
        """Give up the round on every GPU (see NativeStreamingFold.abandon)."""
        for sf in self.folds:
            if sf is not None:
                sf.abandon()

    def finish_device(self, total=None) -> List[torch.Tensor]:
        """Divide on every GPU; the per-GPU bucket results (device tensors)."""
        if self.rows == 0:
            _lib.check(_lib.FA_ERR_NO_CLIENTS, "MultiStreamingFold.finish")
        return [sf.finish(total=total) if sf is not None else None for sf in self.folds]

    def finish(self, total=None) -> np.ndarray:
        """The [P] float32 model in page-locked host memory."""
        accs = self.finish_device(total)
        host = torch.empty(self.P, dtype=torch.float32, pin_memory=True)
        for acc, dev, (lo, hi) in zip(accs, self.devices, self.bounds):
            if acc is not None:
                with torch.cuda.device(dev):
                    host[lo:hi].copy_(acc, non_blocking=True)  # on that GPU's current stream
        for dev in dict.fromkeys(self.devices):
            torch.cuda.current_stream(dev).synchronize()
        return host.numpy()


def scatter_columns(X, devices: Sequence, dtype=None) -> List[torch.Tensor]:
    """Host (numpy or CPU tensor) [N, P] -> each GPU's column bucket [N, P_g] on
    that GPU (row pitch rounded up to 64 elements, as the engine's layout)."""
    devs = resolve_devices(devices)
    Xt = torch.from_numpy(np.ascontiguousarray(X)) if isinstance(X, np.ndarray) else X
    if dtype is not None:
        Xt = Xt.to(dtype)
    N, P = Xt.shape
    parts = []
    for dev, (lo, hi) in zip(devs, column_buckets(P, len(devs))):
        w = hi - lo
        ld = max(64, ((w + 63) // 64) * 64)
        buf = torch.empty((N, ld), dtype=Xt.dtype, device=dev)
        if w:
            buf[:, :w].copy_(Xt[:, lo:hi])
        parts.append(buf[:, :w])
    return parts


def fold_stacked_multi(parts: Sequence[torch.Tensor], weights: Sequence, scores: Optional[Sequence] = None, *,
                       total=None, out: Optional[torch.Tensor] = None, out_device=None) -> torch.Tensor:
    """The fold of a model whose client updates are already resident on
    several GPUs, one column bucket each (parts[g] = [N, P_g] on its GPU, in
    column order; scatter_columns makes them from a host matrix).

    Each GPU folds its bucket on its current stream (engine.fold_stacked: the
    same kernels as one GPU, all launched before any waits); each bucket is
    then copied into `out` ([sum P_g] float32 on out_device, default the first
    part's GPU) with fa_copy_peer on the producing GPU's stream, and the
    destination stream waits for those copies.  Bit-identical to
    engine.fold_stacked over the whole [N, P] matrix."""
    from . import engine
    if not parts:
        raise ValueError("no parts")
    N = parts[0].shape[0]
    if any(p.dim() != 2 or p.shape[0] != N for p in parts):
        raise InvalidParameterShapeError("every part must be [N, P_g] with the same N")
    if any(p.dtype != torch.float32 for p in parts):
        raise InvalidParameterShapeError("fold_stacked_multi takes float32 parts")
    P = sum(p.shape[1] for p in parts)
    total = sum(weights) if total is None else total
    dst = out.device if out is not None else torch.device(out_device) if out_device is not None else parts[0].device
    if dst.index is None:
        dst = torch.device("cuda", torch.cuda.current_device())
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=dst)
    elif out.numel() != P or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 tensor of {P} elements")
    dst_stream = torch.cuda.current_stream(dst)
    ready = torch.cuda.Event()
    ready.record(dst_stream)  # `out` may be written once the destination stream has reached this point
    locals_ = []
    for p in parts:  # every fold is enqueued before anything waits
        locals_.append(engine.fold_stacked(p, weights, scores, total=total) if p.shape[1] else None)
    L = _lib.load()
    off = 0
    done = []
    for p, res in zip(parts, locals_):
        w = p.shape[1]
        if w:
            src_stream = torch.cuda.current_stream(p.device)
            src_stream.wait_event(ready)
            _lib.check(L.fa_copy_peer(out.data_ptr() + off * 4, dst.index, res.data_ptr(), p.device.index, w * 4,
                                      src_stream.cuda_stream), "fa_copy_peer")
            ev = torch.cuda.Event()
            ev.record(src_stream)
            done.append((ev, res))
        off += w
    # A bucket result may be freed when this returns: its memory goes back to
    # its GPU's caching allocator on the stream that also carries the copy, so
    # nothing can reuse it before the copy has read it.
    for ev, _ in done:
        dst_stream.wait_event(ev)
    return out
