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

import math
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


def tail_shares(rounds: int, tail: float, steps: int = 1) -> List[float]:
    """Round shares whose last `steps` rounds shrink geometrically down to
    `tail` times the full rounds (tail=1: equal rounds; rounds=4, tail=0.25,
    steps=2: [1, 1, 0.5, 0.25]).

    Round k's all-gather runs while round k+1 folds, so only the last round's
    exchange is left exposed after the step's folds: a short last round
    shortens it.  But each gather must also fit behind the NEXT fold, or it is
    exposed instead: with gather/fold time ratio rho per parameter (C4 bf16 on
    8 GPUs ~0.55, C3 fp32 ~0.14, DEFAULT_TAIL), round k+1 should keep at least
    rho of round k's width, hence the geometric steps rather than one cut."""
    if not 0 < tail <= 1:
        raise ValueError("tail must be in (0, 1]")
    steps = max(1, min(int(steps), rounds - 1)) if rounds > 1 else 0
    if steps == 0:
        return [1.0] * rounds
    r = float(tail) ** (1.0 / steps)
    return [1.0] * (rounds - steps) + [r ** (j + 1) for j in range(steps)]


# Default overlap layout per input dtype: (tail, steps) for tail_shares.  Each
# round's all-gather must hide behind the next round's fold, and the last one is
# exposed.  Per parameter, the gather moves (world-1) x the output bytes over
# xGMI while the fold reads N x the input bytes from HBM: at 8 GPUs, ~7 TB/s of
# fold and an assumed ~0.35 TB/s per rank of all-gather give a gather/fold
# time ratio rho ~0.14 for C3 (1024 clients, fp32 out) and ~0.55 for C4 (256
# clients, bf16 in and out).  fp32: one cut, shares 1, 1, 1, 0.125 (round 3's
# gather still hides behind round 4's fold at rho 0.14; the steeper 1, 1,
# 0.35, 0.125 measured 0.11 ms more fold per C3 rank step on one GPU);
# bf16: a gentle geometric tail, 1, 0.7, 0.49, 0.34, so that every round
# still covers the previous round's gather.
DEFAULT_TAIL = {"f32": (0.125, 1), "bf16": (0.343, 3)}


def overlap_layout(P: int, world: int, dtype: str = "f32", rounds: int = 4, align: int = ALIGN,
                   quantum: int = 0) -> "SlotLayout":
    """The SlotLayout ShardedAggregator.aggregate_slots should get for a
    `dtype` ("f32" / "bf16") model of P params over `world` ranks (quantum:
    see SlotLayout, e.g. pass_quantum())."""
    tail, steps = DEFAULT_TAIL[dtype]
    return SlotLayout(P, world, rounds, align=align, shares=tail_shares(rounds, tail, steps) if rounds > 1 else None,
                      quantum=quantum)


def pass_quantum(cus: int, dtype: str = "f32") -> int:
    """Columns one pass of the one-launch step's wide tiles covers (a block per
    CU, 256 lanes x 4 quads / octets): a round that is a whole number of
    passes completes with its last pass instead of a tile-time after it."""
    return cus * 256 * 4 * (8 if dtype == "bf16" else 4)


class SlotLayout:
    """Round-robin parameter slots for an exchange that overlaps the fold.

    The global vector is cut into `rounds` rounds of `world` slots each
    (64-element aligned, the last ones partly or wholly past P).  In round k
    every rank's slot is width(k) elements; slot r of round k belongs to rank
    r, so round k's slots of all ranks form the CONTIGUOUS global range
    round_range(k): one all_gather_into_tensor per round writes it in place,
    while the fold of round k+1 runs.  A rank stores its slots side by side:
    round k at local columns [offset(k), offset(k) + width(k)), local width
    sum(width).  By default every round has the same width `sub` (offset(k) =
    k*sub); `shares` sizes the rounds unequally (tail_shares: a short last
    round, whose exchange is the one the step leaves exposed).  rounds=1 is
    exactly bucket_bounds().
    """

    def __init__(self, P: int, world: int, rounds: int = 1, align: int = ALIGN,
                 shares: Optional[Sequence[float]] = None, quantum: int = 0):
        if world < 1 or rounds < 1:
            raise ValueError("world and rounds must be >= 1")
        self.P, self.world, self.rounds = P, world, rounds
        units = -(-P // align)
        if shares is None or len(set(shares)) <= 1:
            if shares is not None and len(shares) != rounds:
                raise ValueError(f"{len(shares)} shares for {rounds} rounds")
            w = align * -(-units // (world * rounds)) if P else 0
            self.widths = [w] * rounds
        else:
            if len(shares) != rounds or min(shares) <= 0:
                raise ValueError(f"need {rounds} positive shares, got {list(shares)}")
            tot = float(sum(shares))
            # each round's slot rounds UP to whole align units, so the rounds cover [0, P)
            self.widths = [align * math.ceil(units * s / (world * tot)) if P else 0 for s in shares]
            while P and world * sum(self.widths) < align * units:  # float rounding slack
                self.widths[0] += align
        if quantum and rounds > 1 and P:
            # every round but the last a whole number of `quantum` columns (the
            # nearest, at least one), the last round the rest
            if quantum % align:
                raise ValueError(f"quantum {quantum} is not a multiple of align {align}")
            total = sum(self.widths)
            head = [max(quantum, quantum * round(w / quantum)) for w in self.widths[:-1]]
            while sum(head) > total - align:  # the last round keeps at least one align unit
                i = max(range(len(head)), key=lambda j: head[j])
                if head[i] <= quantum:
                    raise ValueError(f"{rounds} rounds of {quantum}-column quanta do not fit {total} columns")
                head[i] -= quantum
            self.widths = head + [total - sum(head)]
        self.sub = self.widths[0]  # the uniform layout's slot width (offset(k) = k*sub there)
        self._offs = [0]
        for w in self.widths:
            self._offs.append(self._offs[-1] + w)
        self.local_width = self._offs[-1]
        self.padded_total = world * self.local_width

    @property
    def uniform(self) -> bool:
        return len(set(self.widths)) <= 1

    def width(self, k: int) -> int:
        return self.widths[k]

    def offset(self, k: int) -> int:
        """Local column of round k's slot in a rank's side-by-side storage."""
        return self._offs[k]

    def slot(self, rank: int, k: int) -> Tuple[int, int]:
        """Global [lo, hi) of rank's k-th slot (clipped to P; may be empty)."""
        lo = self.world * self._offs[k] + rank * self.widths[k]
        return min(self.P, lo), min(self.P, lo + self.widths[k])

    def slots(self, rank: int) -> List[Tuple[int, int]]:
        return [self.slot(rank, k) for k in range(self.rounds)]

    def round_range(self, k: int) -> Tuple[int, int]:
        return self.world * self._offs[k], self.world * self._offs[k + 1]


_fold_streams: dict = {}
_gather_streams: dict = {}


def fold_stream(device) -> torch.cuda.Stream:
    """A high-priority stream per GPU for the folds that overlap the exchange.

    HIP maps streams onto a few hardware queues per device; a fold sharing a
    queue with RCCL's stream waits behind the previous round's collective
    instead of running beside it (profiles/r03_c4_trace/).  A high-priority
    stream sits on its own queue."""
    dev = torch.device(device)
    s = _fold_streams.get(dev)
    if s is None:
        s = _fold_streams[dev] = torch.cuda.Stream(device=dev, priority=-1)
    return s


def gather_stream(device) -> torch.cuda.Stream:
    """The stream a one-launch step issues its exchanges from (behind each
    round's wait, sharding.ShardedAggregator.aggregate_slots)."""
    dev = torch.device(device)
    s = _gather_streams.get(dev)
    if s is None:
        s = _gather_streams[dev] = torch.cuda.Stream(device=dev)
    return s


def gather_into(full: torch.Tensor, piece: torch.Tensor, group, async_op: bool):
    """all_gather_into_tensor of `piece` into `full`.  16-bit payloads travel
    as bytes (bit-identical; an all-gather moves bytes, and gloo takes neither
    bfloat16 nor int16).  Under gloo a device piece is staged through host
    memory (CPU rehearsals only); under nccl this is RCCL over xGMI."""
    if piece.dtype in (torch.bfloat16, torch.float16):
        full, piece = full.view(torch.uint8), piece.view(torch.uint8)
    if piece.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(full.shape, dtype=full.dtype)
        dist.all_gather_into_tensor(host, piece.cpu(), group=group)
        full.copy_(host)
        return None
    return dist.all_gather_into_tensor(full, piece, group=group, async_op=async_op)


class ShardedAggregator:
    """Fold this rank's parameter bucket, then all-gather the global model.

    `fold` maps (X_local [N, P_r], weights, scores, out=, total=, want_bf16=)
    -> [P_r] (or (f32, bf16) with want_bf16 on bf16 input), the contract of
    engine.fold_stacked, which is the default.  Tests on CPU (gloo) pass the
    oracle instead.  `total` is the divisor sum over EVERY weight (the
    reference divides by sum(weights) even where zip() truncated the rows,
    fed_avg_aggregator.py:31-35).
    """

    # calls per step form the "auto" mode times before it keeps the faster
    PROBE_CALLS = 2

    def __init__(self, group: Optional[dist.ProcessGroup] = None, fold: Optional[Callable] = None,
                 one_launch="auto"):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        from . import engine
        self.default_fold = fold is None
        if fold is None:
            fold = engine.fold_stacked
        self.fold = fold
        # aggregate_slots folds every round of a step in one launch
        # (engine.fold_rounds) and starts each round's exchange behind that
        # round's completion flag (True), or one fold launch per round (False);
        # "auto": the first calls of a shape alternate the two, each timed on
        # the device and maxed over the group's ranks, then the faster is kept
        # for the shape (which wins depends on how much the exchange kernels
        # slow the fold on this machine)
        if one_launch not in (True, False, "auto"):
            raise ValueError(f"one_launch must be True, False or 'auto', not {one_launch!r}")
        self.one_launch = one_launch
        self._probe: dict = {}  # shape key -> {"one": [ms], "per": [ms]} while probing, or the chosen bool

    def step_form(self, X_local: torch.Tensor, layout: "SlotLayout") -> Optional[str]:
        """The step form "auto" settled on for this shape ("one launch" /
        "per round"), or None while it is still timing them."""
        got = self._probe.get(self._shape_key(X_local, layout))
        return None if got is None or isinstance(got, dict) else ("one launch" if got else "per round")

    def _shape_key(self, X_local, layout):
        # clients by power-of-two bucket (the count changes from round to round
        # with stragglers; a form's advantage does not), the layout exactly
        n = int(X_local.shape[0])
        return (1 << max(0, n - 1).bit_length(), X_local.dtype, tuple(layout.widths), layout.world, layout.P)

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
            if out.numel() < chunk * self.world or not out.is_contiguous() or out.dtype != local.dtype:
                raise ValueError(f"out needs {chunk * self.world} contiguous {local.dtype} elements")
            full = out[: chunk * self.world]
        else:
            full = torch.empty(chunk * self.world, dtype=local.dtype, device=local.device)
        gather_into(full, padded, self.group, async_op=False)
        return full[:P]

    def aggregate(self, X_local: torch.Tensor, weights: Sequence, scores: Optional[Sequence] = None,
                  P: Optional[int] = None, total=None) -> torch.Tensor:
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
            local = self.fold(X_local, weights, scores, total=total)
        else:
            local = torch.empty(0, dtype=torch.float32, device=X_local.device)
        return self.gather(local, P)

    def aggregate_slots(self, X_local: torch.Tensor, weights: Sequence, scores: Optional[Sequence],
                        layout: "SlotLayout", out: Optional[torch.Tensor] = None, total=None) -> torch.Tensor:
        """Fold round by round and all-gather each round asynchronously, so the
        exchange of round k overlaps the fold of round k+1.

        X_local: [N, layout.local_width], this rank's slots side by side (columns
        past P may hold anything; their outputs are trimmed).  Returns [P]:
        float32 for fp32 updates; for bf16 updates the RNE bf16 model (the fold
        still accumulates in fp32), so the exchange moves 2 bytes per parameter,
        half the xGMI bytes of the fp32 result.  `fold` must accept out= (and
        want_bf16= for bf16 input), as engine.fold_stacked does."""
        if X_local.shape[1] != layout.local_width:
            raise ValueError(f"X_local has {X_local.shape[1]} columns, layout needs {layout.local_width}")
        if not X_local.is_cuda or layout.rounds == 1:
            return self._aggregate_slots(X_local, weights, scores, layout, out, total)
        one = self._one_launch_ok(X_local, weights, scores, layout, total)
        probing = None
        # the probe's schedule and its collective depend only on what every rank
        # shares (the fold, the layout, the client count), never on this rank's
        # own buffers: a rank that cannot take the one launch still times its
        # per-round calls in step with the others
        if self.one_launch == "auto" and self.default_fold and 1 < layout.rounds <= 8:
            key = self._shape_key(X_local, layout)
            if key not in self._probe and len(self._probe) >= 64:  # bounded: forget the oldest shape
                self._probe.pop(next(iter(self._probe)))
            got = self._probe.setdefault(key, {"one": [], "per": []})
            if isinstance(got, dict):  # still timing: the form with fewer timed calls, one launch first
                probing = (key, "one" if len(got["one"]) <= len(got["per"]) else "per")
                one = one and probing[1] == "one"
            else:
                one = one and got
        # the rounds' folds on a high-priority stream of their own (fold_stream), ordered after
        # the caller's work and before the caller's later work
        caller = torch.cuda.current_stream(X_local.device)
        fs = fold_stream(X_local.device)
        fs.wait_stream(caller)
        with torch.cuda.stream(fs):
            if probing:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(fs)
            if one:
                full = self._aggregate_slots_one_launch(X_local, weights, scores, layout, out, total)
            else:
                full = self._aggregate_slots(X_local, weights, scores, layout, out, total)
            if probing:
                ev[1].record(fs)
        caller.wait_stream(fs)
        full.record_stream(caller)
        if probing:
            self._record_probe(probing, ev, X_local.device)
        return full

    def _record_probe(self, probing, ev, device) -> None:
        """One timed call of the "auto" mode: its device time (max over the
        group's ranks, so every rank keeps the same form); after PROBE_CALLS
        calls of each form the faster one (best call) is kept for the shape."""
        key, form = probing
        ev[1].synchronize()
        t = torch.tensor([ev[0].elapsed_time(ev[1])], dtype=torch.float64, device=device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        got = self._probe[key]
        got[form].append(float(t.item()))
        if len(got["one"]) >= self.PROBE_CALLS and len(got["per"]) >= self.PROBE_CALLS:
            self._probe[key] = min(got["one"]) <= min(got["per"])

    def _one_launch_ok(self, X_local, weights, scores, layout, total) -> bool:
        import numpy as np

        from .engine import result_dtype
        if not (self.one_launch is not False and self.default_fold and X_local.is_cuda) or not 1 < layout.rounds <= 8:
            return False
        if X_local.dtype not in (torch.float32, torch.bfloat16) or X_local.stride(1) != 1:
            return False
        if X_local.shape[0] < 1 or min(layout.widths) < 1:
            return False
        align = 8 if X_local.dtype == torch.bfloat16 else 4
        if any(layout.offset(k) % align for k in range(layout.rounds)) or X_local.stride(0) % align:
            return False
        if X_local.data_ptr() % 16:
            return False
        return result_dtype(np.dtype(np.float32), list(weights), scores, total) == np.float32

    def _aggregate_slots_one_launch(self, X_local, weights, scores, layout, out, total):
        """Every round's fold in ONE launch on the current (fold) stream; round
        k's exchange issued on the gather stream behind a wait for round k, so
        it runs while the launch folds the later rounds."""
        from . import engine
        dev = X_local.device
        bf16 = X_local.dtype == torch.bfloat16
        odt = torch.bfloat16 if bf16 else torch.float32
        full = out if out is not None else torch.empty(layout.padded_total, dtype=odt, device=dev)
        if full.dtype != odt or full.numel() < layout.padded_total:
            raise ValueError(f"out needs {layout.padded_total} {odt} elements")
        local = torch.empty(layout.local_width, dtype=torch.float32, device=dev)
        local_b = torch.empty(layout.local_width, dtype=torch.bfloat16, device=dev) if bf16 else None
        offs = [layout.offset(k) for k in range(layout.rounds + 1)]
        r = engine.fold_rounds(X_local, weights, scores, offs, out=local, out_bf16=local_b, total=total)
        fs = torch.cuda.current_stream(dev)
        gs = gather_stream(dev)
        send_all = local_b if bf16 else local
        send_all.record_stream(gs)
        works = []
        for k in range(layout.rounds):
            engine.wait_round(r, k, gs)
            lo, hi = layout.round_range(k)
            send = send_all[layout.offset(k):layout.offset(k + 1)]
            with torch.cuda.stream(gs):
                if self.world == 1:
                    full[lo:hi].copy_(send)
                    continue
                w = gather_into(full[lo:hi], send, self.group, async_op=True)
            if w is not None:
                works.append(w)
        for w in works:
            w.wait()  # the fold stream waits for the collectives
        fs.wait_stream(gs)
        return full[: layout.P]

    def _aggregate_slots(self, X_local, weights, scores, layout, out, total):
        bf16 = X_local.dtype == torch.bfloat16
        odt = torch.bfloat16 if bf16 else torch.float32
        full = out if out is not None else torch.empty(layout.padded_total, dtype=odt, device=X_local.device)
        if full.dtype != odt or full.numel() < layout.padded_total:
            raise ValueError(f"out needs {layout.padded_total} {odt} elements")
        local = torch.empty(layout.local_width, dtype=torch.float32, device=X_local.device)
        local_b = torch.empty(layout.local_width, dtype=torch.bfloat16, device=X_local.device) if bf16 else None
        works = []
        for k in range(layout.rounds):
            a, b = layout.offset(k), layout.offset(k) + layout.width(k)
            piece = local[a:b]
            if b > a:
                if bf16:
                    _, pb = self.fold(X_local[:, a:b], weights, scores, out=piece, total=total, want_bf16=True)
                    local_b[a:b].copy_(pb)
                else:
                    self.fold(X_local[:, a:b], weights, scores, out=piece, total=total)
            send = local_b[a:b] if bf16 else piece
            lo, hi = layout.round_range(k)
            if self.world == 1:
                full[lo:hi].copy_(send)
                continue
            w = gather_into(full[lo:hi], send, self.group, async_op=True)
            if w is not None:
                works.append(w)
        for w in works:
            w.wait()
        return full[: layout.P]

    def aggregate_layers(self, parameters: Sequence[Sequence], weights: Sequence,
                         scores: Optional[Sequence] = None, device=None) -> List:
        """Reference-shaped entry (fed_avg_aggregator.py:24-42 over per-client
        layer lists): every rank sees the same per-client float32 numpy layers
        and copies only the pieces of each layer that fall in its own bucket
        (no full-row concatenation).  zip() truncation is kept: rows beyond the
        shorter of parameters / weights / scores are not folded, but the divisor
        is the sum of every weight.  Other dtypes (float64, integer, mixed) are
        rejected: engine.aggregate_layers handles them on one GPU."""
        import numpy as np

        from .aggregator.exceptions import InvalidParameterShapeError
        from .engine import result_dtype
        n = min(len(parameters), len(weights), len(scores) if scores is not None else len(weights))
        if n == 0:
            return []
        L = min(len(p) for p in parameters[:n])
        shapes = [np.asarray(parameters[0][li]).shape for li in range(L)]
        for i in range(n):
            for li in range(L):
                x = parameters[i][li]
                if not isinstance(x, np.ndarray) or x.dtype != np.float32 or x.shape != shapes[li]:
                    raise InvalidParameterShapeError(
                        f"sharded aggregation takes float32 numpy layers shaped like client 0's; client {i} "
                        f"layer {li} is {getattr(x, 'dtype', type(x))} {getattr(x, 'shape', None)}")
        sc = None if scores is None else list(scores[:n])
        total = sum(weights)
        if result_dtype(np.dtype(np.float32), list(weights), sc, total) != np.float32:
            raise InvalidParameterShapeError("weights/scores promote the float32 layers (numpy scalar types)")
        sizes = [int(np.prod(s)) if len(s) else 1 for s in shapes]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        P = int(offs[-1])
        lo, hi = self.bounds(P)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        host = torch.empty((n, hi - lo), dtype=torch.float32, pin_memory=dev.type == "cuda")
        hv = host.numpy()
        for li in range(L):  # layers overlapping [lo, hi) only
            a, b = max(lo, int(offs[li])), min(hi, int(offs[li + 1]))
            if a >= b:
                continue
            for i in range(n):
                hv[i, a - lo:b - lo] = parameters[i][li].reshape(-1)[a - offs[li]:b - offs[li]]
        X = host.to(dev, non_blocking=True) if dev.type == "cuda" else host
        full = self.aggregate(X, list(weights[:n]), sc, P=P, total=total)
        if full.is_cuda:
            from . import engine
            flat = engine.to_host(full)
        else:
            flat = full.numpy()
        return [flat[offs[li]:offs[li + 1]].reshape(shapes[li]) for li in range(L)]
