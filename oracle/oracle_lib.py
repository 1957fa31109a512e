"""ORACLE — ctypes wrapper of the C restatement (oracle/fedavg_ref.c).

TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).  Builds
oracle/build/liboracle.so on first use if it is missing (gcc is present on
both this container and the GPU box).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_i64 = ctypes.c_int64
_vp = ctypes.c_void_p


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_fedavg_f32.argtypes = [_vp, _i64, _i64, _i64, _vp, _vp, ctypes.c_float, _vp, ctypes.c_int]
        L.oracle_fedavg_f64.argtypes = [_vp, _i64, _i64, _i64, _vp, _vp, ctypes.c_double, _vp, ctypes.c_int]
        L.oracle_fedavg_bf16.argtypes = [_vp, _i64, _i64, _i64, _vp, _vp, ctypes.c_float, _vp, _vp, ctypes.c_int]
        L.oracle_synth_f32.argtypes = [_vp, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, ctypes.c_int]
        L.oracle_synth_bf16.argtypes = [_vp, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, ctypes.c_int]
        L.oracle_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_vp) if a is not None else None


def fedavg_f32(X: np.ndarray, a: np.ndarray, divisor: float, s: np.ndarray | None = None,
               nthreads: int = 0) -> np.ndarray:
    assert X.dtype == np.float32 and X.ndim == 2 and X.strides[1] == 4
    N, P = X.shape
    ldx = X.strides[0] // 4
    a = np.ascontiguousarray(a, dtype=np.float32)
    s = None if s is None else np.ascontiguousarray(s, dtype=np.float32)
    out = np.empty(P, dtype=np.float32)
    lib().oracle_fedavg_f32(_p(X), N, P, ldx, _p(a), _p(s), float(np.float32(divisor)), _p(out), nthreads)
    return out


def fedavg_f64(X: np.ndarray, a: np.ndarray, divisor: float, s: np.ndarray | None = None,
               nthreads: int = 0) -> np.ndarray:
    assert X.dtype == np.float64 and X.ndim == 2 and X.strides[1] == 8
    N, P = X.shape
    a = np.ascontiguousarray(a, dtype=np.float64)
    s = None if s is None else np.ascontiguousarray(s, dtype=np.float64)
    out = np.empty(P, dtype=np.float64)
    lib().oracle_fedavg_f64(_p(X), N, P, X.strides[0] // 8, _p(a), _p(s), float(divisor), _p(out), nthreads)
    return out


def fedavg_bf16(Xbits: np.ndarray, a, divisor, s=None, nthreads: int = 0):
    assert Xbits.dtype == np.uint16 and Xbits.ndim == 2 and Xbits.strides[1] == 2
    N, P = Xbits.shape
    a = np.ascontiguousarray(a, dtype=np.float32)
    s = None if s is None else np.ascontiguousarray(s, dtype=np.float32)
    out = np.empty(P, dtype=np.float32)
    outb = np.empty(P, dtype=np.uint16)
    lib().oracle_fedavg_bf16(_p(Xbits), N, P, Xbits.strides[0] // 2, _p(a), _p(s),
                             float(np.float32(divisor)), _p(out), _p(outb), nthreads)
    return out, outb


def synth_f32(seed: int, nrows: int, ncols: int, row0: int = 0, col0: int = 0, nthreads: int = 0):
    X = np.empty((nrows, ncols), dtype=np.float32)
    lib().oracle_synth_f32(_p(X), nrows, ncols, ncols, seed, row0, col0, nthreads)
    return X


def synth_bf16(seed: int, nrows: int, ncols: int, row0: int = 0, col0: int = 0, nthreads: int = 0):
    X = np.empty((nrows, ncols), dtype=np.uint16)
    lib().oracle_synth_bf16(_p(X), nrows, ncols, ncols, seed, row0, col0, nthreads)
    return X


def max_threads() -> int:
    return lib().oracle_max_threads()
