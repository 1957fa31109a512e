"""ctypes binding of libfedavg_hip.so (declarations: include/fedavg_hip.h).

No fallback: if the library is missing or a call fails, this raises.  The
product path never computes an aggregate on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

from .aggregator.exceptions import (
    AggregationError,
    InsufficientClientResults,
    InvalidParameterShapeError,
)

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_PATH = os.path.join(PKG, "_native", "libfedavg_hip.so")
HEADER = os.path.join(REPO, "include", "fedavg_hip.h")
ABI_VERSION = 1

FA_OK, FA_ERR_ARG, FA_ERR_NO_CLIENTS, FA_ERR_SHAPE, FA_ERR_HIP = range(5)

_i64 = ctypes.c_int64
_vp = ctypes.c_void_p
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_int = ctypes.c_int

# name -> (restype, argtypes); must cover every function declared in the header
_PROTOS = {
    "fa_abi_version": (_int, []),
    "fa_last_error": (ctypes.c_char_p, []),
    "fa_fedavg_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp]),
    "fa_fedavg_f32_ptrs": (_int, [_vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp]),
    "fa_fedavg_f32_ptrs_aligned": (_int, [_vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp]),
    "fa_fedavg_f32_splitn": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp]),
    "fa_fold_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _f32, _int, _vp, _vp]),
    "fa_accumulate_f32": (_int, [_vp, _vp, _f32, _f32, _int, _i64, _vp]),
    "fa_finalize_f32": (_int, [_vp, _f32, _vp, _i64, _vp]),
    "fa_fedavg_bf16": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp]),
    "fa_fedavg_f64": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f64, _vp, _vp]),
    "fa_fedavg_i32": (_int, [_vp, _i64, _i64, _i64, _vp, _f64, _vp, _vp]),
    "fa_fedavg_i64": (_int, [_vp, _i64, _i64, _i64, _vp, _f64, _vp, _vp]),
    "fa_synth_f32": (_int, [_vp, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, _vp]),
    "fa_synth_bf16": (_int, [_vp, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, _vp]),
    "fa_read_sweep_f32": (_int, [_vp, _i64, _vp, _i64, _vp]),
    "fa_fedavg_f32_variant": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int]),
    "fa_num_variants": (_int, []),
    "fa_variant_name": (ctypes.c_char_p, [_int]),
    "fa_fedavg_bf16_variant": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _int]),
    "fa_num_bf16_variants": (_int, []),
    "fa_bf16_variant_name": (ctypes.c_char_p, [_int]),
    "fa_npz_index": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _int]),
    "fa_pack": (_int, [_vp, _vp, _vp, _vp, _i64, _int]),
    "fa_bson_elements": (_i64, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64]),
    "fa_bson_walk": (_i64, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64]),
    "fa_host_is_pinned": (_int, [_vp, _i64]),
    "fa_host_alloc": (_int, [_vp, _i64]),
    "fa_host_free": (_int, [_vp]),
    "fa_copy_h2d": (_int, [_vp, _vp, _i64, _vp]),
}

_lock = threading.Lock()
_lib = None


def header_functions() -> list[str]:
    """Every `fa_*(` function declared in include/fedavg_hip.h."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", text)))


def load(path: str | None = None):
    """Load and type the library (idempotent).  Raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise AggregationError(
                f"HIP extension not built: {p} missing (run `python -m fedlesscan_amd.native_build`)")
        L = ctypes.CDLL(p)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        v = L.fa_abi_version()
        if v != ABI_VERSION:
            raise AggregationError(f"libfedavg_hip ABI {v} != expected {ABI_VERSION}")
        _lib = L
        return L


def last_error() -> str:
    return load().fa_last_error().decode(errors="replace")


def check(rc: int, what: str) -> None:
    """Map a C-ABI status onto the reference's exception classes."""
    if rc == FA_OK:
        return
    msg = f"{what}: {last_error()}"
    if rc == FA_ERR_NO_CLIENTS:
        raise InsufficientClientResults(msg)
    if rc == FA_ERR_SHAPE:
        raise InvalidParameterShapeError(msg)
    if rc == FA_ERR_ARG:
        raise ValueError(msg)
    raise AggregationError(msg)


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)
