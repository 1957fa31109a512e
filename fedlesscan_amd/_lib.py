"""ctypes binding of libfedavg_hip.so (declarations: include/fedavg_hip.h)
and of the bench / tuning library libfedavg_hip_bench.so
(include/fedavg_hip_bench.h), which only bench.py and the tests load.

No fallback: if the library is missing or a call fails, this raises.  The
product path never computes an aggregate on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import re
import sysconfig
import threading

from .aggregator.exceptions import (
    AggregationError,
    InsufficientClientResults,
    InvalidParameterShapeError,
)

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_PATH = os.path.join(PKG, "_native", "libfedavg_hip.so")
BENCH_LIB_PATH = os.path.join(PKG, "_native", "libfedavg_hip_bench.so")
# host-only CPython helper (csrc/hostfast.c), built next to the libraries
HOSTFAST_PATH = os.path.join(PKG, "_native", "_hostfast" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
HEADER = os.path.join(REPO, "include", "fedavg_hip.h")
BENCH_HEADER = os.path.join(REPO, "include", "fedavg_hip_bench.h")
ABI_VERSION = 6

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
    "fa_fedavg_f32_hostf": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp]),
    "fa_fedavg_f32_ptrs_hostf": (_int, [_vp, _i64, _i64, _vp, _vp, _f32, _int, _vp, _vp]),
    "fa_fedavg_bf16_hostf": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp]),
    "fa_factors_fill": (_int, [_vp, _vp, _vp, _i64, _vp]),
    "fa_fedavg_f32_splitn": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp]),
    "fa_fold_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _f32, _int, _vp, _vp]),
    "fa_accumulate_f32": (_int, [_vp, _vp, _f32, _f32, _int, _i64, _vp]),
    "fa_finalize_f32": (_int, [_vp, _f32, _vp, _i64, _vp]),
    "fa_fedavg_bf16": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp]),
    "fa_rounds_create": (_int, [_vp, _int]),
    "fa_rounds_destroy": (_int, [_vp]),
    "fa_fedavg_f32_rounds": (_int, [_vp, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _int, _vp, _vp, _vp]),
    "fa_fedavg_bf16_rounds": (_int, [_vp, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int, _vp, _vp, _vp]),
    "fa_fedavg_f32_rounds_hostf": (_int, [_vp, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _int, _vp, _vp, _vp]),
    "fa_fedavg_bf16_rounds_hostf": (_int, [_vp, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int, _vp, _vp, _vp]),
    "fa_rounds_wait": (_int, [_vp, _int, _vp]),
    "fa_rounds_check": (_int, [_vp]),
    "fa_rounds_timeouts": (_int, [_vp]),
    "fa_rounds_form": (ctypes.c_char_p, [_int]),
    "fa_peers_create": (_int, [_vp, _int, _int, _int, _i64]),
    "fa_peers_destroy": (_int, [_vp]),
    "fa_peers_handle_bytes": (_int, []),
    "fa_peers_handle": (_int, [_vp, _vp]),
    "fa_peers_open": (_int, [_vp, _vp]),
    "fa_peers_send": (_vp, [_vp]),
    "fa_peers_rounds": (_vp, [_vp]),
    "fa_peers_exchange": (_int, [_vp, _int, _vp, _vp, _vp, _vp]),
    "fa_fedavg_f64": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f64, _vp, _vp]),
    "fa_fedavg_i32": (_int, [_vp, _i64, _i64, _i64, _vp, _f64, _vp, _vp]),
    "fa_fedavg_i64": (_int, [_vp, _i64, _i64, _i64, _vp, _f64, _vp, _vp]),
    "fa_npz_index": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _int]),
    "fa_crc32": (_int, [_vp, _i64, ctypes.c_uint32, _int, ctypes.POINTER(ctypes.c_uint32)]),
    "fa_pack": (_int, [_vp, _vp, _vp, _vp, _i64, _int]),
    "fa_bson_elements": (_i64, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64]),
    "fa_bson_walk": (_i64, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64]),
    "fa_host_is_pinned": (_int, [_vp, _i64]),
    "fa_host_alloc": (_int, [_vp, _i64]),
    "fa_host_free": (_int, [_vp]),
    "fa_copy_h2d": (_int, [_vp, _vp, _i64, _vp]),
    "fa_copy_peer": (_int, [_vp, _int, _vp, _int, _i64, _vp]),
    "fa_set_autotune": (_int, [_int]),
    "fa_autotune_pending": (_int, []),
    "fa_fold_form": (ctypes.c_char_p, [_int, _i64, _i64, _i64, _int, _vp]),
    "fa_tune_cache_path": (_int, [ctypes.c_char_p]),
    "fa_tune_export": (_i64, [_vp, _i64]),
    "fa_tune_import": (_int, [ctypes.c_char_p]),
    "fa_step_lookup": (_int, [ctypes.c_char_p]),
    "fa_step_record": (_int, [ctypes.c_char_p, _int]),
    "fa_ingest_create": (_int, [_vp, _i64, _i64, _int, _int]),
    "fa_ingest_rows_per_chunk": (_int, [_vp]),
    "fa_ingest_begin": (_int, [_vp, _vp, _vp, _i64]),
    "fa_ingest_add": (_int, [_vp, _vp, _vp, _i64, _f32, _f32, _int]),
    "fa_ingest_finish": (_int, [_vp, _f32]),
    "fa_ingest_destroy": (_int, [_vp]),
}

# libfedavg_hip_bench.so (include/fedavg_hip_bench.h)
_BENCH_PROTOS = {
    "fa_bench_last_error": (ctypes.c_char_p, []),
    "fa_synth_f32": (_int, [_vp, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, _vp]),
    "fa_synth_bf16": (_int, [_vp, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, _vp]),
    "fa_read_sweep_f32": (_int, [_vp, _i64, _vp, _i64, _vp]),
    "fa_bench_copy_f32": (_int, [_vp, _vp, _i64, _int, _vp]),
    "fa_bench_stream_cu_mask": (_int, [_int, _vp, _int, _vp]),
    "fa_bench_stream_destroy": (_int, [_vp]),
    "fa_fedavg_f32_variant": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int]),
    "fa_num_variants": (_int, []),
    "fa_variant_name": (ctypes.c_char_p, [_int]),
    "fa_f32_pick_name": (ctypes.c_char_p, [_i64, _i64, _i64]),
    "fa_num_f32_forms": (_int, []),
    "fa_f32_form_name": (ctypes.c_char_p, [_int]),
    "fa_fedavg_f32_form": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int]),
    "fa_num_ptrs_forms": (_int, []),
    "fa_ptrs_form_name": (ctypes.c_char_p, [_int]),
    "fa_fedavg_f32_ptrs_form": (_int, [_vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int]),
    "fa_num_bf16_forms": (_int, []),
    "fa_bf16_form_name": (ctypes.c_char_p, [_int]),
    "fa_fedavg_bf16_form": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _int]),
    "fa_fedavg_bf16_variant": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _int]),
    "fa_num_bf16_variants": (_int, []),
    "fa_bf16_variant_name": (ctypes.c_char_p, [_int]),
    "fa_fedavg_f32_ptrs_variant": (_int, [_vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int]),
    "fa_num_step_forms": (_int, []),
    "fa_step_form_name": (ctypes.c_char_p, [_int]),
    "fa_bench_rounds_create": (_int, [_vp, _int]),
    "fa_bench_rounds_destroy": (_int, [_vp]),
    "fa_fedavg_rounds_form": (_int, [_vp, _int, _vp, _i64, _i64, _vp, _vp, _f32, _vp, _vp, _int, _vp, _vp]),
    "fa_bench_rounds_wait": (_int, [_vp, _int, _vp]),
    "fa_bench_rounds_set_sys": (_int, [_vp, _int]),
    "fa_num_ptrs_variants": (_int, []),
    "fa_ptrs_variant_name": (ctypes.c_char_p, [_int]),
}

_lock = threading.Lock()
_lib = None
_bench = None


def header_functions(header: str = HEADER) -> list[str]:
    """Every `fa_*(` function declared in a header (default include/fedavg_hip.h)."""
    with open(header) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", text)))


def _open(p: str, protos: dict):
    if not os.path.exists(p):
        raise AggregationError(
            f"HIP extension not built: {p} missing (run `python -m fedlesscan_amd.native_build`)")
    L = ctypes.CDLL(p)
    for name, (res, args) in protos.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def load(path: str | None = None):
    """Load and type the product library (idempotent).  Raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        L = _open(path or LIB_PATH, _PROTOS)
        v = L.fa_abi_version()
        if v != ABI_VERSION:
            raise AggregationError(f"libfedavg_hip ABI {v} != expected {ABI_VERSION}")
        _lib = L
        return L


def load_bench(path: str | None = None):
    """Load and type the bench / tuning library (bench.py and tests only)."""
    global _bench
    with _lock:
        if _bench is None:
            _bench = _open(path or BENCH_LIB_PATH, _BENCH_PROTOS)
        return _bench


def last_error() -> str:
    return load().fa_last_error().decode(errors="replace")


def check(rc: int, what: str, bench: bool = False) -> None:
    """Map a C-ABI status onto the reference's exception classes.  bench=True:
    the status came from libfedavg_hip_bench.so (its own error string)."""
    if rc == FA_OK:
        return
    err = load_bench().fa_bench_last_error().decode(errors="replace") if bench else last_error()
    msg = f"{what}: {err}"
    if rc == FA_ERR_NO_CLIENTS:
        raise InsufficientClientResults(msg)
    if rc == FA_ERR_SHAPE:
        raise InvalidParameterShapeError(msg)
    if rc == FA_ERR_ARG:
        raise ValueError(msg)
    raise AggregationError(msg)


def tune_export() -> str:
    """This process's measured form choices, as tuner cache-file lines."""
    L = load()
    n = L.fa_tune_export(None, 0)
    buf = ctypes.create_string_buffer(int(n) + 1)
    L.fa_tune_export(buf, n + 1)
    return buf.value.decode()


def tune_import(text: str) -> int:
    """Apply tuner cache-file lines (e.g. rank 0's choices); returns how many applied."""
    n = load().fa_tune_import(text.encode())
    if n < 0:
        check(n, "fa_tune_import")
    return int(n)


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)
