"""Device-side aggregation engine: numpy-exact scalar factors + HIP folds.

Layering
  engine.fold_stacked(X, weights, scores)   X: CUDA tensor [N, P] (row pitch = X.stride(0))
  engine.fold_rows(rows, weights, scores)   N separately allocated CUDA rows (pointer list;
                                            engine.RowSet prepares a reusable row set)
  engine.aggregate_layers(params, weights)  host or device per-client layer lists -> per-layer outputs

The scalar factors are formed on the host exactly as numpy forms them in the
reference (fed_avg_aggregator.py:31-41, stall_aware_aggregation.py:52-66):
Python-scalar weights are *weak* (rounded once to the array dtype), the total
is a Python ``sum`` (exact for ints), scores are Python floats from a double
division.  The kernels then fold in client order with separate roundings.

There is no CPU fallback anywhere in this module: every output element is
computed by libfedavg_hip.so on the GPU, or the call raises.
"""
from __future__ import annotations

import ctypes
import operator
import os
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .aggregator.exceptions import InvalidParameterShapeError

_TORCH_TO_NP = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32,
                torch.int64: np.int64, torch.float16: np.float16}
_NP_TO_TORCH = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
                np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64}
ROW_ALIGN = 64  # elements; row pitch multiple of 256 B for fp32


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("fedlesscan_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def result_dtype(in_dtype: np.dtype, weights: Sequence, scores: Optional[Sequence] = None,
                 total=None) -> np.dtype:
    """dtype numpy gives `reduce(add, [x * n_i (* s_i)]) / sum(n)` (NEP 50 weak Python scalars)."""
    in_dtype = np.dtype(in_dtype)
    if in_dtype.kind == "f":
        # Python bool / int / float scalars are weak: a float array keeps its dtype
        kinds = set(map(type, weights))
        if scores is not None:
            kinds.update(map(type, scores))
        if total is not None:
            kinds.add(type(total))
        if kinds <= {bool, int, float}:
            return in_dtype
    if total is None:
        total = sum(weights)
    dt = np.result_type(in_dtype, *weights, *(scores or ()), total)
    if dt.kind in "iu" or dt.kind == "b":
        dt = np.result_type(dt, np.float64)  # true_divide of integers
    return dt


_EXACT_F64 = float(2 ** 53)


def _load_hostfast():
    """The optional CPython helper built next to the HIP libraries (hostfast.c);
    None when it is absent (the numpy path below gives the same bits)."""
    if not os.path.exists(_lib.HOSTFAST_PATH):
        return None
    from importlib.util import module_from_spec, spec_from_file_location
    spec = spec_from_file_location("_hostfast", _lib.HOSTFAST_PATH)
    mod = module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_hostfast = _load_hostfast()


def weak_f32(values) -> Optional[np.ndarray]:
    """np.float32 roundings of `values` when every item is exactly a Python
    bool, int (|v| < 2**53) or float -- numpy's weak scalars, which keep a
    float32 fold float32 -- in one C loop; None otherwise (or without the
    helper), for the general path: result_dtype + round_scalars."""
    if _hostfast is None:
        return None
    b = _hostfast.round_weak_f32(values)
    return None if b is None else np.frombuffer(b, dtype=np.float32)


def round_scalars(values: Sequence, dt: np.dtype) -> np.ndarray:
    """[dt(v) for v in values] -- numpy's rounding of Python (or numpy) scalars
    to `dt`, vectorised.  Going through float64 first is exact whenever every
    value is representable there (ints below 2**53, any float), so rounding the
    float64 array once gives the same bits as rounding each scalar; anything
    else takes the per-element loop."""
    dt = np.dtype(dt)
    try:
        v = (values.astype(np.float64) if isinstance(values, np.ndarray)
             else np.fromiter(values, dtype=np.float64, count=len(values)))
    except (TypeError, ValueError, OverflowError):
        v = None
    if v is not None and v.ndim == 1 and dt.kind == "f" and not (v.size and np.abs(v).max() >= _EXACT_F64):
        return v.astype(dt)
    return np.array([dt.type(x) for x in values], dtype=dt)


class _FactorRing:
    """Page-locked staging slots for the per-client factors of one device: the
    factors of a call travel in ONE async H2D on the caller's stream (instead
    of synchronous pageable copies).  A slot is rewritten only after the copy
    that last read it has completed (its event)."""

    SLOTS, SLOT_BYTES = 8, 1 << 17

    def __init__(self):
        self.host = [torch.empty(self.SLOT_BYTES, dtype=torch.uint8, pin_memory=True) for _ in range(self.SLOTS)]
        self.done = [None] * self.SLOTS
        self.k = 0
        self.lock = threading.Lock()  # callers on several threads share the ring

    def stage(self, parts: List[np.ndarray], dev: torch.device) -> List[torch.Tensor]:
        nbytes = sum(p.nbytes for p in parts)
        if nbytes > self.SLOT_BYTES:  # very many clients: plain copies
            return [torch.from_numpy(np.ascontiguousarray(p)).to(dev) for p in parts]
        with self.lock:
            k = self.k
            self.k = (k + 1) % self.SLOTS
            if self.done[k] is not None:
                self.done[k].synchronize()
            hv = self.host[k].numpy()
            off = 0
            for p in parts:
                hv[off:off + p.nbytes] = np.ascontiguousarray(p).view(np.uint8).reshape(-1)
                off += p.nbytes
            d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            d.copy_(self.host[k][:nbytes], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self.done[k] = ev
        out, off = [], 0
        for p in parts:
            out.append(d[off:off + p.nbytes].view(_NP_TO_TORCH[p.dtype]))
            off += p.nbytes
        return out


_rings: dict = {}
_rings_lock = threading.Lock()


def stage_factors(parts: List[np.ndarray], dev: torch.device) -> List[torch.Tensor]:
    ring = _rings.get(dev)
    if ring is None:
        with _rings_lock:
            ring = _rings.setdefault(dev, None) or _FactorRing()
            _rings[dev] = ring
    return ring.stage(parts, dev)


class Factors:
    """a_i, s_i and the divisor as numpy would round them for compute dtype `dt`."""

    def __init__(self, weights: Sequence, scores: Optional[Sequence], dt: np.dtype, int_weights=False,
                 total=None):
        self.total = sum(weights) if total is None else total
        if int_weights:
            self.a = np.asarray([int(w) for w in weights], dtype=np.int64)
            self.div = float(self.total)
        else:
            self.a = round_scalars(weights, dt)
            self.div = np.dtype(dt).type(self.total)
        self.s = None if scores is None else round_scalars(scores, dt)

    @classmethod
    def weak_f32(cls, weights: Sequence, scores: Optional[Sequence], total=None) -> Optional["Factors"]:
        """Factors of a float32 fold whose weights, scores and total are all
        weak Python scalars (the reference's cardinalities and scores are):
        the result dtype is float32 without a type scan and the rounding is
        one C loop.  None when any value is something else."""
        if total is not None and type(total) not in (bool, int, float):
            return None
        a = weak_f32(weights)
        if a is None:
            return None
        s = None
        if scores is not None:
            s = weak_f32(scores)
            if s is None:
                return None
        f = cls.__new__(cls)
        f.total = sum(weights) if total is None else total
        f.a, f.s = a, s
        f.div = np.float32(f.total)
        return f

    def host(self):
        """(a, s) as host addresses for the *_hostf entries (s: None)."""
        return self.a.ctypes.data, (None if self.s is None else self.s.ctypes.data)

    def to(self, device):
        parts = [self.a] if self.s is None else [self.a, self.s]
        staged = stage_factors(parts, device)
        return staged[0], (staged[1] if self.s is not None else None)


def _captured_factors(f: Factors, dev) -> tuple:
    """Under a HIP graph capture: the float32 factors (a, s or None) in a
    tensor allocated inside the capture -- memory the graph owns -- written by
    fill kernels that carry the values in their arguments (fa_factors_fill),
    for the device-factor entries; the _hostf entries refuse capture."""
    n = len(f.a)
    buf = torch.empty(n * (1 if f.s is None else 2), dtype=torch.float32, device=dev)
    _lib.call("fa_factors_fill", buf.data_ptr(), *f.host(), n, stream_ptr(dev))
    return buf[:n], (None if f.s is None else buf[n:])


def _check_matrix(X: torch.Tensor) -> tuple[int, int, int]:
    if not X.is_cuda:
        raise ValueError("X must be a CUDA (HIP) tensor")
    if X.dim() != 2 or X.stride(1) != 1:
        raise InvalidParameterShapeError(f"X must be 2-D with unit column stride, got {tuple(X.shape)} "
                                         f"strides {X.stride()}")
    N, P = X.shape
    return N, P, X.stride(0) if N > 1 else max(P, 1)


def fold_stacked(X: torch.Tensor, weights: Sequence, scores: Optional[Sequence] = None, *,
                 out: Optional[torch.Tensor] = None, want_bf16: bool = False, total=None,
                 exact: bool = True, out_bf16: Optional[torch.Tensor] = None):
    """FedAvg (scores None) / stall-aware fold over the rows of X, in row order.

    `total` overrides the divisor sum (used when zip() truncated the rows but
    the reference still divides by the sum of every weight).  Returns `out`
    ([P] tensor in the result dtype).  bf16 input: want_bf16=True returns
    (out_f32, out_bf16); out_bf16= (a [P] bfloat16 tensor) receives the RNE
    copy in place -- without out it is the only output (no fp32 result is
    stored, ABI 5) and is returned alone, with out the pair is returned.
    exact=False (fp32 only) opts into the split-client fold,
    fa_fedavg_f32_splitn: faster on very narrow models, deterministic, but NOT
    bit-identical to the reference (a different association of the same sum).
    """
    N, P, ldx = _check_matrix(X)
    if len(weights) != N or (scores is not None and len(scores) != N):
        raise InvalidParameterShapeError(f"{N} rows but {len(weights)} weights"
                                         + ("" if scores is None else f" / {len(scores)} scores"))
    dev = X.device
    st = stream_ptr(dev)
    if out_bf16 is not None and X.dtype != torch.bfloat16:
        raise InvalidParameterShapeError("out_bf16 is for bfloat16 rows")
    if X.dtype == torch.bfloat16:
        f = Factors.weak_f32(weights, scores, total) or Factors(weights, scores, np.dtype(np.float32), total=total)
        if out_bf16 is not None:
            if not (out_bf16.is_cuda and out_bf16.dtype == torch.bfloat16 and out_bf16.is_contiguous()
                    and out_bf16.numel() >= P):
                raise ValueError(f"out_bf16 must be a contiguous CUDA bfloat16 tensor of >= {P} elements")
            outb = out_bf16
        else:
            outb = torch.empty(P, dtype=torch.bfloat16, device=dev) if want_bf16 else None
        if out is None and (outb is None or want_bf16):
            out = torch.empty(P, dtype=torch.float32, device=dev)
        if torch.cuda.is_current_stream_capturing():
            a, s = _captured_factors(f, dev)
            _lib.call("fa_fedavg_bf16", X.data_ptr(), N, P, ldx, a.data_ptr(), _ptr(s), float(f.div),
                      _ptr(out), _ptr(outb), st)
        else:
            _lib.call("fa_fedavg_bf16_hostf", X.data_ptr(), N, P, ldx, *f.host(), float(f.div),
                      _ptr(out), _ptr(outb), st)
        if want_bf16:
            return out, outb
        if out_bf16 is not None:
            return outb if out is None else (out, outb)
        return out
    in_dt = np.dtype(_TORCH_TO_NP.get(X.dtype, np.void))
    if in_dt == np.void:
        raise InvalidParameterShapeError(f"unsupported dtype {X.dtype}")
    # the common case (float32 layers, Python-number weights) skips the type scan
    fw = Factors.weak_f32(weights, scores, total) if in_dt == np.float32 else None
    dt = np.dtype(np.float32) if fw is not None else result_dtype(in_dt, weights, scores, total)
    int_path = in_dt.kind == "i" and scores is None and all(isinstance(w, int) for w in weights)
    if int_path:
        f = Factors(weights, None, dt, int_weights=True, total=total)
        a, _ = f.to(dev)
        out = out if out is not None else torch.empty(P, dtype=torch.float64, device=dev)
        name = "fa_fedavg_i32" if in_dt == np.int32 else "fa_fedavg_i64"
        _lib.call(name, X.data_ptr(), N, P, ldx, a.data_ptr(), f.div, out.data_ptr(), st)
        return out
    if dt not in (np.float32, np.float64):
        raise InvalidParameterShapeError(f"unsupported result dtype {dt} (input {in_dt})")
    if in_dt != dt:
        # numpy promotes the operand before multiplying; same on the device.
        X = X.to(_NP_TO_TORCH[dt])
        ldx = X.stride(0) if N > 1 else max(P, 1)
    f = fw or Factors(weights, scores, dt, total=total)
    out = out if out is not None else torch.empty(P, dtype=_NP_TO_TORCH[dt], device=dev)
    if dt == np.float32:
        # the split-client kernel needs 16-B aligned rows; any other layout
        # takes the exact fold, which is bit-identical to the reference
        split = not exact and X.data_ptr() % 16 == 0 and ldx % 4 == 0 and out.data_ptr() % 16 == 0
        if split:
            a, s = f.to(dev)
            _lib.call("fa_fedavg_f32_splitn", X.data_ptr(), N, P, ldx, a.data_ptr(), _ptr(s), float(f.div),
                      out.data_ptr(), st)
        elif torch.cuda.is_current_stream_capturing():
            a, s = _captured_factors(f, dev)
            _lib.call("fa_fedavg_f32", X.data_ptr(), N, P, ldx, a.data_ptr(), _ptr(s), float(f.div),
                      out.data_ptr(), st)
        else:  # factors from host memory: the library stages them (one C call)
            _lib.call("fa_fedavg_f32_hostf", X.data_ptr(), N, P, ldx, *f.host(), float(f.div), out.data_ptr(), st)
    else:
        a, s = f.to(dev)
        _lib.call("fa_fedavg_f64", X.data_ptr(), N, P, ldx, a.data_ptr(), _ptr(s), float(f.div),
                  out.data_ptr(), st)
    return out


_rounds_states: dict = {}
_rounds_lock = threading.Lock()


def rounds_state(device: torch.device, stream: Optional[int] = None) -> ctypes.c_void_p:
    """The library's one-launch-per-step state (fa_rounds) for the launches
    issued on one stream of a device (default: its current stream), kept for
    the life of the process (torch's streams come from fixed pools, so the
    handles a process sees are few).  Launches with one state must not
    overlap: the library orders each launch after the previous launch of its
    state (an event), so even a stream handle reused after its stream was
    destroyed cannot run two launches of one state at once."""
    dev = torch.device(device)
    key = (dev, stream if stream is not None else stream_ptr(dev))
    with _rounds_lock:
        h = _rounds_states.get(key)
        if h is None:
            h = ctypes.c_void_p()
            _lib.call("fa_rounds_create", ctypes.byref(h), dev.index if dev.index is not None else 0)
            _rounds_states[key] = h
        return h


def f32_factors(weights: Sequence, scores: Optional[Sequence] = None, total=None) -> Optional[Factors]:
    """The float32 factors of a fold over float32 (or bf16) rows, or None when
    numpy would promote the result (numpy-scalar weights, scores or total):
    the weak-scalar fast path first, the type scan only when it declines."""
    f = Factors.weak_f32(weights, scores, total)
    if f is not None:
        return f
    if result_dtype(np.dtype(np.float32), list(weights), scores, total) != np.float32:
        return None
    return Factors(weights, scores, np.dtype(np.float32), total=total)


class StagedFactors:
    """Float32 factors uploaded ONCE (one H2D on the current stream) for the
    several folds of one exchange step (fold_staged): the per-round launches
    of ShardedAggregator read them instead of staging their own per launch."""

    def __init__(self, f: Factors, device):
        self.a, self.s = f.to(torch.device(device))
        self.div = float(f.div)
        self.n = len(f.a)


def fold_staged(X: torch.Tensor, sf: StagedFactors, *, out: Optional[torch.Tensor] = None,
                out_bf16: Optional[torch.Tensor] = None):
    """fold_stacked with staged float32 factors: fp32 rows into out; bf16 rows
    into out and/or out_bf16 (ABI 5).  Returns out (fp32) or out_bf16 when it
    is the only output, else (out, out_bf16)."""
    N, P, ldx = _check_matrix(X)
    if N != sf.n:
        raise InvalidParameterShapeError(f"{N} rows but {sf.n} staged factors")
    st = stream_ptr(X.device)
    for name, t, dt in (("out", out, torch.float32), ("out_bf16", out_bf16, torch.bfloat16)):
        if t is not None and not (t.is_cuda and t.dtype == dt and t.is_contiguous() and t.numel() >= P):
            raise ValueError(f"{name} must be a contiguous CUDA {dt} tensor of >= {P} elements")
    if X.dtype == torch.bfloat16:
        if out is None and out_bf16 is None:
            raise ValueError("fold_staged: bf16 rows need out or out_bf16")
        _lib.call("fa_fedavg_bf16", X.data_ptr(), N, P, ldx, sf.a.data_ptr(), _ptr(sf.s), sf.div, _ptr(out),
                  _ptr(out_bf16), st)
        return out_bf16 if out is None else (out if out_bf16 is None else (out, out_bf16))
    if X.dtype != torch.float32 or out is None or out_bf16 is not None:
        raise ValueError("fold_staged: fp32 rows fold into out (float32), no out_bf16")
    _lib.call("fa_fedavg_f32", X.data_ptr(), N, P, ldx, sf.a.data_ptr(), _ptr(sf.s), sf.div, out.data_ptr(), st)
    return out


def fold_rounds(X: torch.Tensor, weights: Sequence, scores: Optional[Sequence], offsets: Sequence[int], *,
                out=None, out_bf16=None, total=None, state: Optional[ctypes.c_void_p] = None,
                capacity: Optional[int] = None, factors: Optional[Factors] = None,
                out_offsets: Optional[Sequence[int]] = None) -> ctypes.c_void_p:
    """Every exchange round of a step in ONE launch (fa_fedavg_*_rounds): round
    k folds the columns [offsets[k], offsets[k+1]) of X (fp32 or bf16 rows)
    into the same columns of out (fp32) and, for bf16 X, of out_bf16 (the RNE
    copy), on the current stream.  fp32 X needs out; bf16 X needs out,
    out_bf16 or both (ABI 5: a step that exchanges the bf16 copy stores no
    fp32 result).  Returns the rounds state for `wait_round` (the current
    stream's, or `state`: a peer exchange's, fa_peers_rounds): the exchange of
    round k may start, on another stream, as soon as round k is complete,
    while the launch goes on.  Same bits as fold_stacked on each round's
    columns.  out / out_bf16: tensors (at least offsets[-1] elements) or raw
    device addresses (a peer exchange's send buffer), which need `capacity`,
    the elements the address holds.  factors: f32_factors(weights, scores,
    total) when the caller has them already (one step, one rounding).
    out_offsets: round k's results go to output columns [out_offsets[k],
    out_offsets[k] + width k) instead (a rank's slots straight into its chunk
    of the gathered model: the all-gather then runs in place)."""
    N, W, ldx = _check_matrix(X)
    if len(weights) != N or (scores is not None and len(scores) != N):
        raise InvalidParameterShapeError(f"{N} rows but {len(weights)} weights")
    rounds = len(offsets) - 1
    if out_offsets is not None:
        if len(out_offsets) < rounds:
            raise ValueError(f"{len(out_offsets)} output offsets for {rounds} rounds")
        end = max((int(out_offsets[k]) + int(offsets[k + 1]) - int(offsets[k]) for k in range(rounds)), default=0)
    else:
        end = int(offsets[-1]) if len(offsets) else 0
    for name, t, dt in (("out", out, torch.float32), ("out_bf16", out_bf16, torch.bfloat16)):
        if t is None:
            continue
        if isinstance(t, int):
            if capacity is None or end > capacity:
                raise ValueError(f"{name}: a raw address needs capacity >= {end} elements (got {capacity})")
        elif not (t.is_cuda and t.dtype == dt and t.is_contiguous() and t.numel() >= end):
            raise ValueError(f"{name} must be a contiguous CUDA {dt} tensor of >= {end} elements")
    if out is None and (X.dtype != torch.bfloat16 or out_bf16 is None):
        raise ValueError("fold_rounds needs out (fp32 rows) or out / out_bf16 (bf16 rows)")
    dev = X.device
    f = factors if factors is not None else f32_factors(weights, scores, total)
    if f is None:
        raise InvalidParameterShapeError("the rounds fold takes float32 factors (Python-number weights)")
    offs = (ctypes.c_int64 * len(offsets))(*[int(o) for o in offsets])
    oo = None if out_offsets is None else (ctypes.c_int64 * rounds)(*[int(o) for o in out_offsets[:rounds]])
    st = stream_ptr(dev)
    r = state if state is not None else rounds_state(dev, st)
    addr = (lambda t: None if t is None else (t if isinstance(t, int) else t.data_ptr()))
    # the factors from host memory: the library stages them (one C call, _hostf)
    if X.dtype == torch.bfloat16:
        _lib.call("fa_fedavg_bf16_rounds_hostf", r, X.data_ptr(), N, ldx, *f.host(), float(f.div),
                  addr(out), addr(out_bf16), rounds, offs, oo, st)
    elif X.dtype == torch.float32:
        _lib.call("fa_fedavg_f32_rounds_hostf", r, X.data_ptr(), N, ldx, *f.host(), float(f.div),
                  addr(out), rounds, offs, oo, st)
    else:
        raise InvalidParameterShapeError(f"the rounds fold takes float32 or bfloat16 rows, got {X.dtype}")
    return r


def wait_round(state: ctypes.c_void_p, k: int, stream: torch.cuda.Stream) -> None:
    """Enqueue on `stream` a wait for round k of the last fold_rounds launch."""
    _lib.call("fa_rounds_wait", state, int(k), stream.cuda_stream)


def _equal_stride_view(rows, host_ptrs: np.ndarray, P: int) -> Optional[torch.Tensor]:
    """[N, P] view when the fp32 rows sit in ONE storage at a constant forward pitch.

    A device-resident simulation usually hands over `X[i]` rows of one stacked
    tensor (or equal-size slices of one buffer): then the stacked fold reads
    them with ldx = pitch, with no pointer table to build and upload and with
    the narrow-model (LDS-staged) kernels the pointer-list fold lacks.

    Only the first and the last row are asked for their storage: when both lie
    in one storage, every row between them at the constant pitch lies in that
    storage's contiguous range too, so the view reads exactly the bytes the
    rows' own pointers name (as_strided re-checks the bounds)."""
    N = len(rows)
    if N < 2 or P == 0:
        return None
    step = int(host_ptrs[1] - host_ptrs[0])
    if step < P * 4 or step % 4:
        return None
    if (np.diff(host_ptrs) != step).any():
        return None
    base, last = rows[0], rows[-1]
    if last.untyped_storage().data_ptr() != base.untyped_storage().data_ptr():
        return None
    return base.as_strided((N, P), (step // 4, 1))


_dtype_of = operator.attrgetter("dtype")


class RowSet:
    """N client rows already on the GPU, prepared once for repeated folds.

    A device-resident simulation keeps each client's update in its own
    persistent tensor and refolds the same rows every round.  Building a
    RowSet validates the rows and looks at their placement ONCE:
      - rows of one allocation at a constant forward pitch (X[i] of a stacked
        tensor) become one [N, P] strided view: the stacked fold, no table;
      - other fp32 rows get a device table of row pointers for
        fa_fedavg_f32_ptrs_aligned (every row 16-B aligned) or
        fa_fedavg_f32_ptrs (any alignment).
    fold_rows(rowset, weights) then costs the factor upload and the kernel.
    The RowSet keeps the tensors alive; their CONTENTS may change between
    folds, their storage may not (re-create the RowSet after reallocating)."""

    def __init__(self, rows: Sequence[torch.Tensor]):
        rows = list(rows)
        N = len(rows)
        if N == 0:
            _lib.check(_lib.FA_ERR_NO_CLIENTS, "RowSet")
        r0 = rows[0]
        P, dev, dt = r0.numel(), r0.device, r0.dtype
        if not r0.is_cuda:
            raise ValueError("rows must be CUDA (HIP) tensors")
        # one C-level pass per property (a Python loop over 1024 rows with a
        # reshape per row cost ~1 ms per call, more than the fold of 1024 x 67K)
        if (set(map(torch.Tensor.numel, rows)) != {P} or set(map(_dtype_of, rows)) != {dt}
                or not all(map(torch.Tensor.is_contiguous, rows))
                or set(map(torch.Tensor.get_device, rows)) != {r0.get_device()}):
            raise InvalidParameterShapeError("all rows must be contiguous with equal size, dtype, device")
        self.rows = rows
        self.N, self.P, self.device, self.dtype = N, P, dev, dt
        self.view = None
        self.ptrs = None
        self.host_ptrs = None
        self.aligned = False
        if dt == torch.float32 and P > 0:
            host_ptrs = self.host_ptrs = np.fromiter(map(torch.Tensor.data_ptr, rows), dtype=np.int64, count=N)
            self.view = _equal_stride_view(rows, host_ptrs, P)
            if self.view is None:
                self.ptrs = torch.from_numpy(host_ptrs).to(dev)
                self.aligned = not (host_ptrs % 16).any()

    def overlaps(self, t: torch.Tensor) -> bool:
        """Does tensor t share a byte with any row?"""
        if self.host_ptrs is None or self.P == 0 or t.numel() == 0:
            return False
        lo = t.data_ptr()
        hi = lo + t.numel() * t.element_size()
        return bool(np.any((self.host_ptrs < hi) & (lo < self.host_ptrs + self.P * 4)))

    def stacked(self) -> torch.Tensor:
        """The rows copied into one [N, P] tensor (the non-fp32 fallbacks)."""
        return torch.stack([r.reshape(-1) for r in self.rows])


def fold_rows(rows, weights: Sequence, scores: Optional[Sequence] = None, *,
              out: Optional[torch.Tensor] = None, total=None) -> torch.Tensor:
    """The fold over separately allocated 1-D CUDA rows (no stacking copy for
    fp32).  `rows` is a RowSet (prepared once, reusable) or a sequence of
    tensors (a RowSet is built for this call)."""
    rs = rows if isinstance(rows, RowSet) else RowSet(rows)
    if len(weights) != rs.N or (scores is not None and len(scores) != rs.N):
        raise InvalidParameterShapeError(f"{rs.N} rows but {len(weights)} weights"
                                         + ("" if scores is None else f" / {len(scores)} scores"))
    fw = Factors.weak_f32(weights, scores, total) if rs.dtype == torch.float32 else None
    if fw is None and (rs.dtype != torch.float32
                       or result_dtype(np.dtype(np.float32), weights, scores, total) != np.float32):
        return fold_stacked(rs.stacked(), weights, scores, out=out, total=total)
    if rs.view is not None or rs.P == 0:
        # rows of one allocation at a fixed pitch: the stacked fold, no pointer table
        X = rs.view if rs.view is not None else rs.stacked()
        return fold_stacked(X, weights, scores, out=out, total=total)
    dev = rs.device
    f = fw or Factors(weights, scores, np.dtype(np.float32), total=total)
    dst = out
    if out is not None and rs.overlaps(out):
        # out over a client row: the row table lives in device memory, so the
        # library cannot see the alias, and the tuner's first call of a shape
        # runs several launches into out (a later one would read what an earlier
        # wrote).  Fold into a fresh buffer, then copy.
        out = None
    out = out if out is not None else torch.empty(rs.P, dtype=torch.float32, device=dev)
    aligned = rs.aligned and out.data_ptr() % 16 == 0
    if torch.cuda.is_current_stream_capturing():
        a, s = _captured_factors(f, dev)
        _lib.call("fa_fedavg_f32_ptrs_aligned" if aligned else "fa_fedavg_f32_ptrs", rs.ptrs.data_ptr(), rs.N, rs.P,
                  a.data_ptr(), _ptr(s), float(f.div), out.data_ptr(), stream_ptr(dev))
    else:
        _lib.call("fa_fedavg_f32_ptrs_hostf", rs.ptrs.data_ptr(), rs.N, rs.P, *f.host(), float(f.div),
                  int(aligned), out.data_ptr(), stream_ptr(dev))
    if dst is not None and dst is not out:
        dst.copy_(out)
        return dst
    return out


# ---------------------------------------------------------------------------
# per-layer (reference-shaped) aggregation
# ---------------------------------------------------------------------------
def _layer_meta(parameters, n_eff):
    L = min(len(p) for p in parameters[:n_eff])
    shapes, dtypes = [], []
    for li in range(L):
        ref = parameters[0][li]
        shp = tuple(ref.shape)
        dt = ref.dtype
        for ci in range(1, n_eff):
            x = parameters[ci][li]
            if tuple(x.shape) != shp:
                raise InvalidParameterShapeError(
                    f"layer {li}: client {ci} has shape {tuple(x.shape)}, client 0 has {shp}")
            if x.dtype != dt:
                raise InvalidParameterShapeError(f"layer {li}: client {ci} dtype {x.dtype} != {dt}")
        shapes.append(shp)
        dtypes.append(dt)
    return L, shapes, dtypes


def _multi(devices) -> Optional[list]:
    """The device list of a multi-GPU call, or None for a one-GPU call."""
    if devices is None:
        return None
    from .multigpu import resolve_devices
    devs = resolve_devices(devices)
    return devs if len(devs) > 1 else None


def aggregate_layers(parameters: Sequence[Sequence], weights: Sequence, scores: Optional[Sequence] = None,
                     device: Optional[torch.device] = None, devices=None) -> List:
    """Reference-shaped FedAvg / stall-aware aggregation.

    parameters: N clients x L layers (numpy arrays, or CUDA tensors).  Returns
    L outputs (numpy in -> numpy out, tensors in -> CUDA tensors out).  zip()
    truncation over clients/weights/scores and over layers is kept
    (fed_avg_aggregator.py:32-41); the divisor is the sum of ALL weights.

    devices: several GPUs of this process (multigpu.py): host float32 layers
    are folded one column bucket per GPU, bit-identical to one GPU.  Other
    layer groups (device tensors, other dtypes) run on the first of them.
    """
    multi = _multi(devices)
    if multi is not None and device is None:
        device = multi[0]
    elif devices is not None and multi is None and device is None:
        from .multigpu import resolve_devices
        device = resolve_devices(devices)[0]
    n_eff = min(len(parameters), len(weights), len(scores) if scores is not None else len(weights))
    if n_eff == 0:
        return []
    total_weights = list(weights)
    L, shapes, dtypes = _layer_meta(parameters, n_eff)
    if L == 0:
        return []
    on_device = isinstance(parameters[0][0], torch.Tensor)
    dev = device or (parameters[0][0].device if on_device else default_device())
    w = list(weights[:n_eff])
    sc = None if scores is None else list(scores[:n_eff])
    groups: dict = {}
    for li, dt in enumerate(dtypes):
        groups.setdefault(str(dt), []).append(li)
    outs: list = [None] * L
    for _, lis in groups.items():
        sizes = [int(np.prod(shapes[li])) if len(shapes[li]) else 1 for li in lis]
        P = sum(sizes)
        fp32_result = result_dtype(np.dtype(np.float32), total_weights, sc) == np.float32
        if (not on_device and P > 0 and dtypes[lis[0]] == np.float32 and fp32_result):
            # host fp32 rows: pipelined pinned-chunk H2D + in-order chunked fold (bit-identical)
            if multi is not None:  # one column bucket per GPU, result assembled in pinned host memory
                flat = _stream_group_multi(parameters, n_eff, lis, P, w, sc, sum(total_weights), multi)
                off = 0
                for li, n in zip(lis, sizes):
                    outs[li] = flat[off:off + n].reshape(shapes[li])
                    off += n
                continue
            res = _stream_group(parameters, n_eff, lis, P, w, sc, sum(total_weights), dev)
        elif on_device and dtypes[lis[0]] == torch.float32 and fp32_result and all(
                parameters[i][li].is_contiguous() for i in range(n_eff) for li in lis):
            # device fp32 layers: fold each layer straight from the clients' own
            # tensors through a row-pointer list -- no stacking copy
            for li in lis:
                rows = [parameters[i][li].reshape(-1) for i in range(n_eff)]
                outs[li] = fold_rows(rows, w, sc, total=sum(total_weights)).reshape(shapes[li])
            continue
        else:
            X = _stack_group(parameters, n_eff, lis, sizes, P, dev, on_device)
            res = fold_stacked(X, w, sc, total=sum(total_weights))
        flat = res if on_device else to_host(res)
        off = 0
        for li, n in zip(lis, sizes):
            outs[li] = flat[off:off + n].reshape(shapes[li])
            off += n
    return outs


# pinned staging per chunk; FEDAVG_STREAM_CHUNK_MB overrides.  The native pipe
# (ingest.NativeStreamingFold, round 3) keeps 3 chunks of 32 MB in flight: best
# or within the run-to-run spread of 16-64 MB x 3-6 slots on 10 x 582K, 100 x 1M,
# 100 x 10M and 1024 x 1M (profiles/r03_e2e_ramp/); the Python-driven
# StreamingFold (the direct-DMA route) keeps 2.
STREAM_CHUNK_BYTES = int(os.environ.get("FEDAVG_STREAM_CHUNK_MB", "32")) << 20
# DMA layers straight from page-locked documents instead of packing them
# (StreamingFold direct=True); FEDAVG_DIRECT_DMA=1 turns it on.
DIRECT_DMA = os.environ.get("FEDAVG_DIRECT_DMA", "0") == "1"


def _py_scalar(x) -> bool:
    return type(x) in (int, float)  # weak scalars: fp32 layers stay fp32 (NEP 50)


def _fast_row(layers, shapes) -> bool:
    """A row the streaming path can take: float32 numpy layers shaped like row 0."""
    return (len(layers) == len(shapes) and
            all(isinstance(x, np.ndarray) and x.dtype == np.float32 and x.shape == shp
                for x, shp in zip(layers, shapes)))


def aggregate_decoded(items, scores: Optional[Sequence] = None, device: Optional[torch.device] = None,
                      devices=None, expected_rows: int = 0) -> List:
    """aggregate_layers over an iterator of decoded (layers, weight) rows, with
    the fold overlapping the decode.

    The strategies' aggregate() decodes every result and then folds
    (fed_avg_aggregator.py:64-92).  Here each host float32 row enters the
    pipelined StreamingFold as soon as it is decoded, so decoding row i+1
    overlaps the DMA of row i.  Same rows, same order, same factors: the result
    is bit-identical.  Anything else (other dtypes, a row shaped unlike row 0,
    weights that are not Python scalars, device tensors, nothing to fold)
    drains the iterator and runs aggregate_layers over every row, which is
    exactly the materialised path.  zip() truncation is kept: rows beyond
    len(scores) are not folded, their weights still count in the divisor.

    devices: several GPUs (multigpu.MultiStreamingFold): every GPU ingests and
    folds its own column bucket of each row, so the rows cross G PCIe links.
    expected_rows: the number of rows when the caller knows it (a list of
    results); the native pipe then shrinks its last chunks (a shorter tail).
    """
    multi = _multi(devices)
    if devices is not None and device is None:
        from .multigpu import resolve_devices
        device = resolve_devices(devices)[0]
    it = iter(items)
    first = next(it, None)
    if first is None:
        return []
    rows, weights = [first[0]], [first[1]]
    shapes = [getattr(x, "shape", None) for x in first[0]]
    n_fold = len(scores) if scores is not None else None
    fast = (len(shapes) > 0 and _fast_row(first[0], shapes) and _py_scalar(first[1]) and
            (scores is None or (len(scores) > 0 and all(_py_scalar(x) for x in scores))))
    P = sum(int(np.prod(shp)) if len(shp) else 1 for shp in shapes) if fast else 0
    if fast and P > 0:
        n_exp = min(expected_rows, n_fold) if n_fold is not None else expected_rows
        if multi is not None:
            from .multigpu import MultiStreamingFold
            sf = MultiStreamingFold(P, multi, chunk_bytes=STREAM_CHUNK_BYTES, direct=DIRECT_DMA,
                                    expected_rows=n_exp)
        else:
            from .ingest import make_streaming_fold
            sf = make_streaming_fold(P, device or default_device(), STREAM_CHUNK_BYTES, direct=DIRECT_DMA,
                                     expected_rows=n_exp)
        sf.add(list(first[0]), first[1], None if scores is None else scores[0])
        for layers, w in it:
            rows.append(layers)
            weights.append(w)
            i = len(rows) - 1
            if not _py_scalar(w):
                break
            if n_fold is not None and i >= n_fold:
                continue
            if not _fast_row(layers, shapes):
                break
            sf.add(list(layers), w, None if scores is None else scores[i])
        else:
            res = sf.finish(total=sum(weights))
            flat = res if multi is not None else to_host(res)
            outs, off = [], 0
            for shp in shapes:
                n = int(np.prod(shp)) if len(shp) else 1
                outs.append(flat[off:off + n].reshape(shp))
                off += n
            return outs
        sf.abandon()  # release the pipe now: no DMA or fold left running for GC to join
    for layers, w in it:
        rows.append(layers)
        weights.append(w)
    return aggregate_layers(rows, weights, scores, device=device, devices=devices)


def to_host(t: torch.Tensor) -> np.ndarray:
    """D2H of a result through page-locked memory (a pageable .cpu() ran at
    ~7 GB/s, pinned at PCIe rate).  The array views the pinned buffer and keeps
    it alive; the copy runs on the producing stream and is waited for here."""
    host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    host.copy_(t, non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return host.numpy()


def _stream_group(parameters, n, lis, P, w, sc, total, dev) -> torch.Tensor:
    from .ingest import chunk_class, make_streaming_fold
    sf = make_streaming_fold(P, dev, chunk_class(max(1, n) * 4 * P, STREAM_CHUNK_BYTES), direct=DIRECT_DMA,
                             expected_rows=n)
    for i in range(n):
        sf.add([parameters[i][li] for li in lis], w[i], None if sc is None else sc[i])
    return sf.finish(total=total)


def _stream_group_multi(parameters, n, lis, P, w, sc, total, devices) -> np.ndarray:
    from .multigpu import MultiStreamingFold
    sf = MultiStreamingFold(P, devices, chunk_bytes=STREAM_CHUNK_BYTES, direct=DIRECT_DMA, expected_rows=n)
    for i in range(n):
        sf.add([parameters[i][li] for li in lis], w[i], None if sc is None else sc[i])
    return sf.finish(total=total)


def _stack_group(parameters, n, lis, sizes, P, dev, on_device) -> torch.Tensor:
    ldx = ((P + ROW_ALIGN - 1) // ROW_ALIGN) * ROW_ALIGN
    if on_device:
        ref = parameters[0][lis[0]]
        X = torch.empty((n, ldx), dtype=ref.dtype, device=dev)
        for i in range(n):
            off = 0
            for li, sz in zip(lis, sizes):
                X[i, off:off + sz].copy_(parameters[i][li].reshape(-1))
                off += sz
        return X[:, :P]
    np_dt = np.asarray(parameters[0][lis[0]]).dtype
    tdt = _NP_TO_TORCH.get(np_dt)
    if tdt is None:
        raise InvalidParameterShapeError(f"unsupported parameter dtype {np_dt}")
    stage = torch.empty((n, ldx), dtype=tdt, pin_memory=True)
    sv = stage.numpy()
    for i in range(n):
        off = 0
        for li, sz in zip(lis, sizes):
            sv[i, off:off + sz] = np.asarray(parameters[i][li]).reshape(-1)
            off += sz
    X = torch.empty((n, ldx), dtype=tdt, device=dev)
    X.copy_(stage, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()  # stage may be freed after return
    return X[:, :P]
