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
import socket
import warnings
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


def _timing_pair(stream, folds):
    """Two timing events around one fold launch on `stream`, the first recorded
    now and both appended to `folds`; None when folds is None (not timed)."""
    if folds is None:
        return None
    e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    e[0].record(stream)
    folds.append(e)
    return e


def device_ident(device) -> str:
    """The identity a step-form decision is keyed by: gfx arch and CU count of
    `device` ("gfx950:256"), as the tuner's cache file keys kernel forms."""
    p = torch.cuda.get_device_properties(torch.device(device))
    arch = getattr(p, "gcnArchName", "") or p.name
    return f"{arch}:{p.multi_processor_count}".replace(" ", "_")


def step_key(ident: str, bf16: bool, n_clients: int, layout: "SlotLayout", exchange: str = "rccl") -> str:
    """The key of a step-form decision (fa_step_lookup / fa_step_record):
    device identity, dtype (".peer" appended for the peer-copy exchange),
    world size, client-count bucket (the count moves from round to round with
    stragglers; a form's advantage does not), P and the layout's slot widths."""
    bucket = 1 << max(0, int(n_clients) - 1).bit_length()
    dt = ("bf16" if bf16 else "f32") + (".peer" if exchange == "peer_copy" else "")
    return f"{ident} {dt} {layout.world} {bucket} {layout.P} {','.join(str(w) for w in layout.widths)}"


class PeerExchange:
    """The kernel-free exchange of one rank (fa_peers, csrc/peer_exchange.hpp)
    for one slot layout and dtype: this rank's two send buffers (step e's fold
    writes its slots into buffer e % 2), its IPC handles all-gathered once over
    the group, and per step the one-launch fold on the exchange's own rounds
    state and copy pulls of every rank's round-k slot as soon as that rank has
    completed round k.  Creating one is a collective."""

    def __init__(self, group, device, layout: "SlotLayout", bf16: bool):
        import ctypes

        from . import _lib
        L = self.L = _lib.load()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = torch.device(device)
        self.layout, self.bf16 = layout, bf16
        eb = 2 if bf16 else 4
        send_bytes = self.send_bytes = -(-layout.local_width * eb // 16) * 16
        self.h = None
        h = ctypes.c_void_p()
        _lib.call("fa_peers_create", ctypes.byref(h), self.device.index, self.world, self.rank, send_bytes)
        try:
            nb = L.fa_peers_handle_bytes()
            mine = (ctypes.c_uint8 * nb)()
            _lib.call("fa_peers_handle", h, mine)
            if self.world > 1:
                every = [None] * self.world
                dist.all_gather_object(every, bytes(mine), group=group)
            else:
                every = [bytes(mine)]
            joined = b"".join(every)
            _lib.call("fa_peers_open", h, ctypes.create_string_buffer(joined, len(joined)))
        except BaseException:
            L.fa_peers_destroy(h)  # what was opened is closed with it
            raise
        self.h = h
        self.state = ctypes.c_void_p(L.fa_peers_rounds(h))
        R = layout.rounds
        self.offsets = [layout.offset(k) for k in range(R + 1)]
        self.src = (ctypes.c_int64 * (R + 1))(*[o * eb for o in self.offsets])
        self.dst = (ctypes.c_int64 * (R * self.world))(
            *[(layout.round_range(k)[0] + q * layout.width(k)) * eb for k in range(R) for q in range(self.world)])

    def step(self, X_local, weights, scores, full, total, fold_stream_, other_stream, factors=None,
             fold_end: Optional[torch.cuda.Event] = None):
        """The fold (every round in one launch) on fold_stream_ into this
        step's send buffer, the exchange on other_stream into `full`, then
        fold_stream_ waits for the exchange; returns (event after the waits,
        state).  A bf16 step stores only the RNE-bf16 result it exchanges
        (ABI 5).  No fence: the library orders the state's next fold after
        this exchange, and the two send buffers alternate (fa_peers_send).
        fold_end: an event recorded on fold_stream_ right after the fold."""
        from . import _lib, engine
        send = int(self.L.fa_peers_send(self.h))  # this step's buffer
        cap = self.send_bytes // (2 if self.bf16 else 4)
        with torch.cuda.stream(fold_stream_):
            if self.bf16:
                engine.fold_rounds(X_local, weights, scores, self.offsets, out_bf16=send, total=total,
                                   state=self.state, capacity=cap, factors=factors)
            else:
                engine.fold_rounds(X_local, weights, scores, self.offsets, out=send, total=total, state=self.state,
                                   capacity=cap, factors=factors)
            if fold_end is not None:
                fold_end.record(fold_stream_)
        _lib.call("fa_peers_exchange", self.h, self.layout.rounds, self.src, full.data_ptr(), self.dst,
                  other_stream.cuda_stream)
        done = torch.cuda.Event()
        done.record(other_stream)
        fold_stream_.wait_stream(other_stream)
        return done, self.state

    def close(self) -> None:
        """Collective: every rank's exchanges are complete before any buffer goes."""
        from . import _lib
        if self.h is None:
            return
        torch.cuda.synchronize(self.device)
        if self.world > 1:
            dist.barrier(group=self.group)
        _lib.call("fa_peers_destroy", self.h)
        self.h = None


class ShardedAggregator:
    """Fold this rank's parameter bucket, then all-gather the global model.

    `fold` maps (X_local [N, P_r], weights, scores, out=, total=, want_bf16=,
    out_bf16=) -> [P_r], the contract of engine.fold_stacked, which is the
    default (bf16 input: want_bf16 -> (f32, bf16); out_bf16 alone -> the bf16
    result only).  Tests on CPU (gloo) pass the oracle instead.  `total` is
    the divisor sum over EVERY weight (the reference divides by sum(weights)
    even where zip() truncated the rows, fed_avg_aggregator.py:31-35).

    one_launch -- how aggregate_slots runs an exchange step's folds:
      True      one launch for every round (engine.fold_rounds), each round's
                exchange started behind that round's completion flag;
      False     one fold launch per round;
      "auto"    the form recorded for this machine and shape (the tuner's
                cache file, fa_step_lookup: a decision a probe made in an
                earlier process or another rank's, imported), per-round
                launches when none is recorded -- never a timing run or a
                synchronisation of its own, so a one-call process (one FaaS
                invocation, aggregation.py:71-75) runs the recorded form from
                its first call.  At world > 1 the group runs RANK 0's record:
                the first call of a shape in a process broadcasts it (one small
                collective per shape and process), so ranks whose cache files
                differ (another node, a concurrent writer) still take one form
                and issue the same collectives;
      "probe"   as "auto", but a shape with no recorded form is timed: its
                first PROBE_STEPS calls alternate the two forms, PROBE_WARM
                untimed calls of each first (first-use costs: the rounds
                state, buffers, the tuner), then PROBE_CALLS timed calls of
                each, back to back as the steps run (no synchronisation per
                call: a call's device time, from its fold stream's start to its
                end on the caller's stream, hides the host's enqueue as steady
                steps do); the call that completes the schedule reads the
                times, takes their MAX over the group's ranks (one
                all-reduce), keeps the form with the faster best call and
                records it (fa_step_record) for later processes.
    Every rank of a group takes the same form: the choice depends only on
    what the ranks share (the constructor's arguments, the layout, the client
    count, rank 0's record), and a rank whose rows cannot take the one launch
    as they are (not 16-B aligned, a row pitch off the octet / quad grid)
    folds an aligned copy of them instead of leaving the form.
    check -- what a one-launch step does about a round wait that timed out (a
      waiter gives up after 30 s, and the exchange behind it then reads an
      unfinished round):
      "sync"      (default) every call waits for its step's waits, reads the
                  timeout record (fa_rounds_check) and, over an all-reduce
                  (MAX) so that every rank agrees, raises AggregationError
                  (exceptions.py:1) instead of returning the model;
      "deferred"  the call returns at once (pipelined steps); check_timeouts()
                  does the same check for every step since the last one and
                  must be called before the results are used.
    device_ident -- the identity decisions are keyed by (default: the GPU's
      arch and CU count, device_ident()).
    exchange -- how a one-launch step reassembles the model:
      "rccl"       (default) one all_gather_into_tensor per round behind its wait
                   (RCCL over xGMI under "nccl": copy kernels on a few CUs);
      "peer_copy"  each rank pulls its peers' finished slots with copy-engine
                   copies through IPC-opened buffers (PeerExchange, fa_peers):
                   no kernel beside the fold but one wave per round that polls
                   the ranks' flags.  Needs every rank on one host (checked
                   once per layout with a collective; otherwise "rccl");
                   one_launch=False keeps per-round launches with RCCL.
                   close() releases the buffers (a collective).
    trace -- None (default), or a list to which every CUDA exchange step
      appends (fold events, end event): timing events around each fold launch
      on the fold stream, and one on the caller's stream after the step
      (bench.py splits a step into fold and exposed exchange with them).

    A bf16 step folds in fp32 and stores only the RNE-bf16 result it exchanges
    (ABI 5: no fp32 result is written, 2 B/param out instead of 6).
    """

    # the "probe" mode, per step form: untimed calls first, then timed calls;
    # PROBE_STEPS calls of a shape in all before it keeps the faster form
    PROBE_WARM = 1
    PROBE_CALLS = 2
    PROBE_STEPS = 2 * (PROBE_WARM + PROBE_CALLS)

    def __init__(self, group: Optional[dist.ProcessGroup] = None, fold: Optional[Callable] = None,
                 one_launch="auto", check: str = "sync", device_ident: Optional[str] = None,
                 exchange: str = "rccl"):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        from . import engine
        self.default_fold = fold is None
        if fold is None:
            fold = engine.fold_stacked
        self.fold = fold
        if one_launch not in (True, False, "auto", "probe"):
            raise ValueError(f"one_launch must be True, False, 'auto' or 'probe', not {one_launch!r}")
        if check not in ("sync", "deferred"):
            raise ValueError(f"check must be 'sync' or 'deferred', not {check!r}")
        if exchange not in ("rccl", "peer_copy"):
            raise ValueError(f"exchange must be 'rccl' or 'peer_copy', not {exchange!r}")
        self.exchange = exchange
        self._peers: dict = {}  # (layout widths, P, world, bf16, device) -> PeerExchange, or None: not every rank can
        self.one_launch = one_launch
        self.check = check
        self.ident = device_ident
        self.trace: Optional[list] = None
        self._probe: dict = {}  # step key -> {"calls": {form: n}, "timed": [(form, start, end)]} while probing
        self.probed: dict = {}  # step key -> the same, for the probes that have decided
        self._steps: dict = {}  # step key -> True (one launch) / False (per round): decided or restored
        self._agreed: set = set()  # step keys whose decision the group has agreed on (world > 1)
        self._nodecision: set = set()  # agreed keys with no decision on rank 0: this rank's file is not read
        self._pending: list = []  # "deferred": (event after the waits, rounds state) per unchecked step

    def step_key(self, X_local: torch.Tensor, layout: "SlotLayout") -> Optional[str]:
        """This call's step-form key (module step_key); None without an
        identity (a CPU tensor and no device_ident given)."""
        ident = self.ident
        if ident is None:
            if not X_local.is_cuda:
                return None
            ident = self.ident = device_ident(X_local.device)
        return step_key(ident, X_local.dtype == torch.bfloat16, int(X_local.shape[0]), layout, self.exchange)

    def step_form(self, X_local: torch.Tensor, layout: "SlotLayout") -> Optional[str]:
        """The recorded step form for this shape ("one launch" / "per round"),
        or None (nothing recorded, or a probe still timing)."""
        key = self.step_key(X_local, layout)
        got = self._lookup(key)
        return None if got is None else ("one launch" if got else "per round")

    def record_step_form(self, X_local: torch.Tensor, layout: "SlotLayout", one_launch: bool) -> None:
        """Record a step form for this shape: in this process and, merged into
        the tuner's cache file, for later ones (fa_step_record)."""
        key = self.step_key(X_local, layout)
        if key is None:
            raise ValueError("no device identity for a CPU tensor: pass device_ident=")
        from . import _lib
        _lib.call("fa_step_record", key.encode(), 1 if one_launch else 0)
        self._steps[key] = bool(one_launch)
        self._nodecision.discard(key)

    def _lookup(self, key: Optional[str]) -> Optional[bool]:
        if key is None:
            return None
        got = self._steps.get(key)
        if got is None and key not in self._nodecision:
            from . import _lib
            v = _lib.load().fa_step_lookup(key.encode())
            if v == -2:
                raise ValueError(f"malformed step key {key!r}")
            if v >= 0:
                got = self._steps[key] = bool(v)
        return got

    def _backend_device(self, device) -> torch.device:
        return torch.device(device) if dist.get_backend(self.group) == "nccl" else torch.device("cpu")

    def _agree(self, key: Optional[str], device) -> None:
        """world > 1: every rank takes rank 0's decision for `key` (one
        broadcast, the first time this process sees the key)."""
        if self.world == 1 or key is None or key in self._agreed:
            return
        got = self._lookup(key)
        t = torch.tensor([-1 if got is None else int(got)], dtype=torch.int32, device=self._backend_device(device))
        src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
        dist.broadcast(t, src=src, group=self.group)
        v = int(t.item())
        self._agreed.add(key)
        if v < 0:
            self._steps.pop(key, None)
            self._nodecision.add(key)
        else:
            self._steps[key] = bool(v)
            self._nodecision.discard(key)

    def _form(self, X_local: torch.Tensor, layout: "SlotLayout"):
        """(one launch?, probing) for a multi-round CUDA step: the same on
        every rank of the group."""
        if self.one_launch in (True, False) or not 1 < layout.rounds <= 8:
            return self.one_launch is True, None
        key = self.step_key(X_local, layout)
        self._agree(key, X_local.device)
        got = self._lookup(key)
        if got is None and self.one_launch == "probe" and self.default_fold:
            if key not in self._probe and len(self._probe) >= 64:  # bounded: forget the oldest shape
                self._probe.pop(next(iter(self._probe)))
            t = self._probe.setdefault(key, {"calls": {"one": 0, "per": 0}, "timed": []})
            # the form with fewer calls, one launch first; a form's first
            # PROBE_WARM calls untimed: the schedule depends only on what every
            # rank shares, so all ranks time the same calls
            n = t["calls"]
            form = "one" if n["one"] <= n["per"] else "per"
            probing = (key, form, n[form] >= self.PROBE_WARM)
            return form == "one", probing
        return bool(got), None

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
        out_bf16= for bf16 input), as engine.fold_stacked does.  Raises
        AggregationError (every rank) when a one-launch step's round wait timed
        out (check="sync"; "deferred": at check_timeouts())."""
        if X_local.shape[1] != layout.local_width:
            raise ValueError(f"X_local has {X_local.shape[1]} columns, layout needs {layout.local_width}")
        if not X_local.is_cuda or torch.cuda.is_current_stream_capturing():
            # CPU ranks, or a HIP graph capture (the one launch refuses
            # capture: its epochs would replay): per-round launches, nothing
            # timed or checked
            return self._aggregate_slots(X_local, weights, scores, layout, out, total)
        # the factors, rounded once for the whole step (numpy's weak-scalar
        # rule, engine.f32_factors): the default fold's slots are float32 /
        # bf16 buffers, so promoted factors (numpy-scalar weights) are refused
        f = None
        if self.default_fold:
            from .aggregator.exceptions import InvalidParameterShapeError
            from .engine import f32_factors
            if X_local.dtype not in (torch.float32, torch.bfloat16):
                raise InvalidParameterShapeError(f"sharded slots take float32 or bfloat16 rows, not {X_local.dtype}")
            f = f32_factors(weights, scores, total)
            if f is None:
                raise InvalidParameterShapeError("weights/scores promote the float32 fold (numpy scalar types)")
        one, probing = self._form(X_local, layout)
        one = one and self._one_launch_ok(X_local, layout)
        # the rounds' folds on a high-priority stream of their own (fold_stream), ordered after
        # the caller's work and before the caller's later work
        dev = X_local.device
        caller = torch.cuda.current_stream(dev)
        fs = fold_stream(dev)
        if caller != fs:  # a caller already on the fold stream needs no hop
            fs.wait_stream(caller)
        timed = probing is not None and probing[2]
        folds = [] if (timed or self.trace is not None) else None  # (start, end) timing events per fold launch
        waited = None
        with torch.cuda.stream(fs):
            if one:
                X_local = self._aligned(X_local)
            px = self._peer_exchange(X_local, layout) if (one and self.exchange == "peer_copy") else None
            if px is not None:
                odt = torch.bfloat16 if px.bf16 else torch.float32
                full = out if out is not None else torch.empty(layout.padded_total, dtype=odt, device=dev)
                if full.dtype != odt or full.numel() < layout.padded_total or not full.is_contiguous():
                    raise ValueError(f"out needs {layout.padded_total} contiguous {odt} elements")
                e = _timing_pair(fs, folds)
                waited = px.step(X_local, weights, scores, full, total, fs, gather_stream(dev), factors=f,
                                 fold_end=None if e is None else e[1])
                full = full[: layout.P]
            elif one:
                full, waited = self._aggregate_slots_one_launch(X_local, weights, scores, layout, out, total, folds, f)
            else:
                full = self._aggregate_slots(X_local, weights, scores, layout, out, total, folds, f)
        if caller != fs:
            caller.wait_stream(fs)
            full.record_stream(caller)
        if folds is not None:
            end = torch.cuda.Event(enable_timing=True)
            end.record(caller)
            if self.trace is not None:
                self.trace.append((folds, end))
        if waited is not None:
            if self.check == "sync":
                waited[0].synchronize()
                self._raise_on_timeouts(self._timed_out([waited[1]]), dev)
            else:
                self._pending.append(waited)
        if probing:
            self._record_probe(probing, folds[0][0] if timed else None, end if timed else None, X_local, layout)
        return full

    def _timed_out(self, states) -> int:
        from . import _lib
        L = _lib.load()
        n = 0
        for st in {id(x): x for x in states}.values():
            v = L.fa_rounds_check(st)
            if v < 0:
                _lib.check(-v, "fa_rounds_check")
            n += v
        return n

    def _raise_on_timeouts(self, n: int, device=None) -> None:
        """Every rank learns whether any rank's round wait timed out (MAX over
        the group) and, if one did, raises: an exchange behind that wait read
        an unfinished round, so no rank may use the gathered model."""
        if self.world > 1:
            dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
            t = torch.tensor([n], dtype=torch.int32, device=self._backend_device(dev))
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            n = int(t.item())
        if n:
            from .aggregator.exceptions import AggregationError
            raise AggregationError(
                f"round wait timed out ({n} round(s) on the worst rank): the exchange read an unfinished round; "
                "the aggregated model is not valid")

    def check_timeouts(self) -> None:
        """check="deferred": wait for every unchecked step's round waits, then
        raise AggregationError on every rank if any of them timed out.  A
        collective over the group: every rank calls it at the same point."""
        pending, self._pending = self._pending, []
        if pending:
            pending[-1][0].synchronize()  # the waits complete in stream order
        self._raise_on_timeouts(self._timed_out([p[1] for p in pending]))

    def close(self) -> None:
        """Release the peer exchanges' buffers (exchange="peer_copy"): a
        collective, after every rank's last step."""
        for px in self._peers.values():
            if px is not None:
                px.close()
        self._peers.clear()

    def _peer_exchange(self, X_local, layout):
        """This layout's PeerExchange, created on first use (a collective: the
        ranks' hosts are compared and their handles all-gathered), or None --
        the RCCL exchange -- when the ranks are not all on one host (IPC
        handles open only on the host that made them)."""
        bf16 = X_local.dtype == torch.bfloat16
        key = (tuple(layout.widths), layout.P, layout.world, bf16, X_local.device)
        if key not in self._peers:
            ok = True
            if self.world > 1:
                hosts = [None] * self.world
                dist.all_gather_object(hosts, socket.gethostname(), group=self.group)
                ok = len(set(hosts)) == 1
            self._peers[key] = PeerExchange(self.group, X_local.device, layout, bf16) if ok else None
        return self._peers[key]

    def _record_probe(self, probing, start, end, X_local, layout) -> None:
        """One call of the "probe" mode: counted, and its (start, end) events
        kept when timed.  The call that completes the schedule reads every
        timed call's device time (waiting for its own end only), takes the MAX
        over the group's ranks (one all-reduce, so every rank keeps the same
        form) and records the form with the faster best call
        (record_step_form: this process and the cache file)."""
        key, form, timed = probing
        got = self._probe[key]
        got["calls"][form] += 1
        if timed:
            got["timed"].append((form, start, end))
        if min(got["calls"].values()) < self.PROBE_WARM + self.PROBE_CALLS:
            return
        del self._probe[key]
        end = got["timed"][-1][2]
        end.synchronize()  # the calls' events complete in stream order
        t = torch.tensor([s.elapsed_time(e) for _, s, e in got["timed"]], dtype=torch.float64,
                         device=self._backend_device(X_local.device) if self.world > 1 else "cpu")
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        ms = [float(x) for x in t.tolist()]
        res = {f: [m for (g, _, _), m in zip(got["timed"], ms) if g == f] for f in ("one", "per")}
        self.probed[key] = res  # what the decision saw (ms per timed call, max over ranks)
        while len(self.probed) > 64:
            self.probed.pop(next(iter(self.probed)))
        self.record_step_form(X_local, layout, min(res["one"]) <= min(res["per"]))

    def _one_launch_ok(self, X_local, layout) -> bool:
        """Can the step run as one launch?  Only what every rank shares (the
        fold, dtype, layout, client count; the factors were checked float32 by
        the caller): a rank's own row alignment is fixed by _aligned, so the
        ranks never split on it."""
        if not (self.default_fold and X_local.is_cuda) or not 1 < layout.rounds <= 8:
            return False
        if X_local.dtype not in (torch.float32, torch.bfloat16):
            return False
        if X_local.shape[0] < 1 or min(layout.widths) < 1:
            return False
        align = 8 if X_local.dtype == torch.bfloat16 else 4
        return not any(layout.offset(k) % align for k in range(layout.rounds))

    @staticmethod
    def _aligned(X_local: torch.Tensor) -> torch.Tensor:
        """X_local, or an aligned copy of it when its rows are not 16-B aligned
        or its pitch is off the octet (bf16) / quad (fp32) grid: the one
        launch's 16-byte loads need both.  The copy runs on the current stream
        (the fold stream), in order before the fold that reads it."""
        align = 8 if X_local.dtype == torch.bfloat16 else 4
        if (X_local.data_ptr() % 16 == 0 and X_local.stride(1) == 1
                and (X_local.shape[0] == 1 or X_local.stride(0) % align == 0)):
            return X_local
        warnings.warn(f"aggregate_slots: rows at {X_local.data_ptr():#x} with pitch {X_local.stride(0)} cannot take "
                      "the one-launch step as they are; folding an aligned copy (allocate X_local 16-B aligned with "
                      f"a pitch that is a multiple of {align} elements to avoid it)", RuntimeWarning, stacklevel=3)
        Y = torch.empty(X_local.shape, dtype=X_local.dtype, device=X_local.device)
        Y.copy_(X_local)
        return Y

    def _own(self, layout: "SlotLayout", k: int) -> Tuple[int, int]:
        """[lo, hi) of this rank's chunk of round k in the gathered model (its
        slot k, padding included): where the fold writes it, so each round's
        all-gather runs in place."""
        lo = layout.round_range(k)[0] + self.rank * layout.width(k)
        return lo, lo + layout.width(k)

    def _aggregate_slots_one_launch(self, X_local, weights, scores, layout, out, total, folds=None, factors=None):
        """Every round's fold in ONE launch on the current (fold) stream, each
        round's slot written straight into this rank's chunk of the model
        (out_offsets); round k's in-place all-gather issued on the gather
        stream behind a wait for round k, so it runs while the launch folds the
        later rounds -- except the last round's, issued on the fold stream
        itself right after the launch (stream order is its wait).  At world 1
        there is nothing to exchange: the launch alone writes the model.
        Returns the model and (an event after the waits, the rounds state) for
        the timeout check, or None when no wait ran or check="sync" already
        checked them (before the last round's gather)."""
        from . import engine
        dev = X_local.device
        bf16 = X_local.dtype == torch.bfloat16
        odt = torch.bfloat16 if bf16 else torch.float32
        full = out if out is not None else torch.empty(layout.padded_total, dtype=odt, device=dev)
        if full.dtype != odt or full.numel() < layout.padded_total or not full.is_contiguous():
            raise ValueError(f"out needs {layout.padded_total} contiguous {odt} elements")
        offs = [layout.offset(k) for k in range(layout.rounds + 1)]
        own = [self._own(layout, k) for k in range(layout.rounds)]
        fs = torch.cuda.current_stream(dev)
        e = _timing_pair(fs, folds)
        # all the fold stores: the fp32 result, or for bf16 rows only its
        # RNE-bf16 copy (no fp32 result, ABI 5) -- the form the exchange moves
        kw = {"out_bf16": full} if bf16 else {"out": full}
        r = engine.fold_rounds(X_local, weights, scores, offs, total=total, factors=factors,
                               out_offsets=[lo for lo, _ in own], **kw)
        if e is not None:
            e[1].record(fs)
        if self.world == 1:
            return full[: layout.P], None
        gs = gather_stream(dev)
        full.record_stream(gs)
        works = []
        waits_done = torch.cuda.Event()
        last = layout.rounds - 1
        waited = (waits_done, r)
        for k in range(layout.rounds):
            lo, hi = layout.round_range(k)
            if k < last:
                engine.wait_round(r, k, gs)
                if k == last - 1:
                    waits_done.record(gs)  # every round's wait has run (the timeout check)
            elif self.check == "sync":
                # check="sync" here, before the last round's gather: the waits
                # (rounds 0..R-2; the last round is ordered by the stream) are
                # done while the launch still folds the last round, and the
                # check's MAX all-reduce goes on the gather stream, ahead of
                # the last gather -- so the host's wait and the collective
                # overlap the fold's tail instead of following the step.  A
                # timeout raises on every rank here, before any rank issues the
                # last gather (the MAX agrees)
                waits_done.synchronize()
                with torch.cuda.stream(gs):
                    self._raise_on_timeouts(self._timed_out([r]), dev)
                waited = None
            with torch.cuda.stream(gs if k < last else fs):
                w = gather_into(full[lo:hi], full[own[k][0]:own[k][1]], self.group, async_op=True)
            if w is not None:
                works.append(w)
        for w in works:
            w.wait()  # the fold stream waits for the collectives
        fs.wait_stream(gs)
        return full[: layout.P], waited

    def _aggregate_slots(self, X_local, weights, scores, layout, out, total, folds=None, factors=None):
        bf16 = X_local.dtype == torch.bfloat16
        odt = torch.bfloat16 if bf16 else torch.float32
        full = out if out is not None else torch.empty(layout.padded_total, dtype=odt, device=X_local.device)
        if full.dtype != odt or full.numel() < layout.padded_total or not full.is_contiguous():
            raise ValueError(f"out needs {layout.padded_total} contiguous {odt} elements")
        # each round's fold writes straight into this rank's chunk of the model
        # (fp32 rows the fp32 result, bf16 rows only its RNE-bf16 copy), and the
        # round's all-gather runs in place: at world 1 nothing is copied
        cur = torch.cuda.current_stream(X_local.device) if X_local.is_cuda else None
        staged = None
        if factors is not None and X_local.is_cuda and not torch.cuda.is_current_stream_capturing():
            # the step's factors uploaded once, for every round's launch
            from .engine import StagedFactors
            staged = StagedFactors(factors, X_local.device)
        works = []
        for k in range(layout.rounds):
            a, b = layout.offset(k), layout.offset(k) + layout.width(k)
            olo, ohi = self._own(layout, k)
            piece = full[olo:ohi]
            if b > a:
                e = _timing_pair(cur, folds) if cur is not None else None
                if staged is not None:
                    from .engine import fold_staged
                    fold_staged(X_local[:, a:b], staged, **({"out_bf16": piece} if bf16 else {"out": piece}))
                elif bf16:
                    self.fold(X_local[:, a:b], weights, scores, out_bf16=piece, total=total)
                else:
                    self.fold(X_local[:, a:b], weights, scores, out=piece, total=total)
                if e is not None:
                    e[1].record(cur)
            if self.world == 1:
                continue
            lo, hi = layout.round_range(k)
            w = gather_into(full[lo:hi], piece, self.group, async_op=True)
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
