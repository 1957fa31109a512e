"""Parameter-bucket sharding across the GPUs of one node.

Every output parameter is independent, so the P columns of the stacked
[N clients x P] update matrix are split into contiguous per-rank buckets; each
rank folds its bucket over ALL N clients locally (no cross-GPU reduction, so
the fold stays bit-exact), and the only exchange is one all-gather of the
per-rank output buckets to reassemble the global model on every rank.  With
the "nccl" backend that all-gather is RCCL over xGMI; under "gloo" (CPU tests)
it is the same call on CPU tensors.

One process per GPU (torch.distributed.run); nothing here assumes a rank
count, so 1/2/4/8 GPUs use the same code.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

ALIGN = 64  # elements: bucket starts stay 256-byte aligned for fp32


def bucket_bounds(P: int, world: int, align: int = ALIGN) -> List[Tuple[int, int]]:
    """[start, end) of every rank's bucket: equal aligned chunks, the tail short.

    All buckets except the last non-empty one are exactly `chunk` long, so the
    rank-ordered concatenation of the padded buckets starts with [0, P)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    units = -(-P // align)
    chunk = align * -(-units // world) if P else 0
    return [(min(P, r * chunk), min(P, (r + 1) * chunk)) for r in range(world)]


def chunk_size(P: int, world: int, align: int = ALIGN) -> int:
    b = bucket_bounds(P, world, align)
    return b[0][1] - b[0][0]


class ShardedAggregator:
    """Fold this rank's parameter bucket, then all-gather the global model.

    `fold` maps (X_local [N, P_r], weights, scores) -> [P_r]; it defaults to
    the HIP engine.  Tests on CPU (gloo) pass the oracle instead.
    """

    def __init__(self, group: Optional[dist.ProcessGroup] = None, fold: Optional[Callable] = None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if fold is None:
            from . import engine
            fold = engine.fold_stacked
        self.fold = fold

    def bounds(self, P: int) -> Tuple[int, int]:
        return bucket_bounds(P, self.world)[self.rank]

    def gather(self, local: torch.Tensor, P: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """All-gather the per-rank buckets into the full [P] model on every rank.

        `out`, if given, must hold world * chunk_size(P, world) elements (the
        padded layout); the gather then writes into it with no extra copy and
        out[:P] is returned."""
        chunk = chunk_size(P, self.world)
        if self.world == 1:
            return local if out is None else out[:P].copy_(local)
        if local.numel() != chunk:
            padded = torch.zeros(chunk, dtype=local.dtype, device=local.device)
            padded[: local.numel()] = local
        else:
            padded = local
        if out is not None:
            if out.numel() < chunk * self.world or not out.is_contiguous():
                raise ValueError(f"out needs {chunk * self.world} contiguous elements")
            full = out[: chunk * self.world]
        else:
            full = torch.empty(chunk * self.world, dtype=local.dtype, device=local.device)
        if padded.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo has no device transport: stage through host memory (rehearsal / no-RCCL hosts)
            host = torch.empty(full.shape, dtype=full.dtype)
            dist.all_gather_into_tensor(host, padded.cpu(), group=self.group)
            full.copy_(host)
        else:
            dist.all_gather_into_tensor(full, padded, group=self.group)
        return full[:P]

    def aggregate(self, X_local: torch.Tensor, weights: Sequence, scores: Optional[Sequence] = None,
                  P: Optional[int] = None) -> torch.Tensor:
        """X_local = this rank's columns [start, end) of the stacked updates, all N clients."""
        if P is None:
            t = torch.tensor([X_local.shape[1]], dtype=torch.int64, device=X_local.device)
            if self.world > 1:
                dist.all_reduce(t, group=self.group)
            P = int(t.item())
        lo, hi = self.bounds(P)
        if X_local.shape[1] != hi - lo:
            raise ValueError(f"rank {self.rank} holds {X_local.shape[1]} columns, bucket is [{lo}, {hi})")
        if hi > lo:
            local = self.fold(X_local, weights, scores)
        else:
            local = torch.empty(0, dtype=torch.float32, device=X_local.device)
        return self.gather(local, P)

    def aggregate_layers(self, parameters: Sequence[Sequence], weights: Sequence,
                         scores: Optional[Sequence] = None, device=None) -> List:
        """Reference-shaped entry: every rank sees the same per-client layer lists
        (numpy) and H2D-copies only its own bucket of each client's row."""
        import numpy as np
        n = min(len(parameters), len(weights), len(scores) if scores is not None else len(weights))
        if n == 0:
            return []
        L = min(len(p) for p in parameters[:n])
        shapes = [np.asarray(parameters[0][li]).shape for li in range(L)]
        sizes = [int(np.prod(s)) if len(s) else 1 for s in shapes]
        P = sum(sizes)
        lo, hi = self.bounds(P)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        dt = np.asarray(parameters[0][0]).dtype
        host = np.empty((n, hi - lo), dtype=dt)
        for i in range(n):
            row = np.concatenate([np.asarray(parameters[i][li]).reshape(-1) for li in range(L)])
            host[i] = row[lo:hi]
        X = torch.from_numpy(host).to(dev)
        full = self.aggregate(X, list(weights[:n]), None if scores is None else list(scores[:n]), P=P)
        flat = full.cpu().numpy()
        outs, off = [], 0
        for shp, sz in zip(shapes, sizes):
            outs.append(flat[off:off + sz].reshape(shp))
            off += sz
        return outs
