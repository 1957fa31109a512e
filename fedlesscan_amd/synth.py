"""Deterministic synthetic client updates (host side, numpy).

The same generator is implemented as a HIP kernel (``fa_synth_*`` in
``csrc/fedavg.hip``).  Every step is integer arithmetic followed by an exact
int->float conversion and a power-of-two scale, so the device and the host
produce *bit-identical* values.  That lets a test regenerate any column slice
of a 41 GB device-resident workload on the host and check it bit-exactly.

Element (row i, column j) of a workload with seed ``seed``::

    key_i  = mix64(seed * GOLDEN ^ mix64(i + 1))
    h      = mix64(key_i + (j + 1) * GOLDEN)
    v      = (h[0:21] + h[21:42] + h[42:63]) - 3 * 2**20      # Irwin-Hall(3), |v| < 2**22
    x[i,j] = float32(v) * 2**-24                             # exact; ~N(0, 0.0625**2)

``mix64`` is the splitmix64 finaliser.  The Irwin-Hall(3) sum stands in for the
Box-Muller draw SURVEY.md 8(d) sketches: transcendental functions are not
bit-reproducible between libm and the device math library, integer sums are.

Per-client cardinalities ``n_i = lo + mix64(seed*GOLDEN ^ mix64(i+1) ^ CARD) % (hi-lo+1)``
and stall-aware round ids are drawn the same way from independent streams.
"""
from __future__ import annotations

import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
CARD_SALT = 0xC2B2AE3D27D4EB4F
ROUND_SALT = 0x165667B19E3779F9

_U = np.uint64
_MASK21 = _U((1 << 21) - 1)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    z ^= z >> _U(30)
    z *= _U(M1)
    z ^= z >> _U(27)
    z *= _U(M2)
    z ^= z >> _U(31)
    return z


def _mix64_int(z: int) -> int:
    m = (1 << 64) - 1
    z &= m
    z ^= z >> 30
    z = (z * M1) & m
    z ^= z >> 27
    z = (z * M2) & m
    z ^= z >> 31
    return z


def row_key(seed: int, row: int) -> int:
    m = (1 << 64) - 1
    return _mix64_int(((seed * GOLDEN) & m) ^ _mix64_int(row + 1))


def client_row_f32(seed: int, row: int, col0: int, ncols: int) -> np.ndarray:
    """Columns [col0, col0+ncols) of client ``row`` as float32."""
    key = _U(row_key(seed, row))
    j = np.arange(col0 + 1, col0 + ncols + 1, dtype=np.uint64)
    h = _mix64(key + j * _U(GOLDEN))
    s = (h & _MASK21) + ((h >> _U(21)) & _MASK21) + ((h >> _U(42)) & _MASK21)
    v = s.astype(np.int64) - 3 * (1 << 20)
    return v.astype(np.float32) * np.float32(2.0 ** -24)


def clients_f32(seed: int, n: int, col0: int, ncols: int, row0: int = 0) -> np.ndarray:
    """[n, ncols] float32 block of rows row0..row0+n-1."""
    out = np.empty((n, ncols), dtype=np.float32)
    for r in range(n):
        out[r] = client_row_f32(seed, row0 + r, col0, ncols)
    return out


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even float32 -> bfloat16 bit pattern (NaN stays NaN)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = (u + _U(0x7FFF) + ((u >> _U(16)) & _U(1))) >> _U(16)
    nan = np.isnan(np.asarray(x, dtype=np.float32))
    r = np.where(nan, (u >> _U(16)) | _U(0x40), r)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def clients_bf16(seed: int, n: int, col0: int, ncols: int, row0: int = 0) -> np.ndarray:
    """[n, ncols] bf16 bit patterns (uint16): RNE of the float32 generator."""
    return f32_to_bf16_bits(clients_f32(seed, n, col0, ncols, row0))


def cardinalities(seed: int, n: int, lo: int = 1, hi: int = 600) -> list[int]:
    m = (1 << 64) - 1
    span = hi - lo + 1
    return [lo + _mix64_int((((seed * GOLDEN) & m) ^ _mix64_int(i + 1)) ^ CARD_SALT) % span
            for i in range(n)]


def round_ids(seed: int, n: int, current_round: int, tolerance: int) -> list[int]:
    """Result round ids in [R - tolerance, R] (FedLesScan stale-result window)."""
    m = (1 << 64) - 1
    span = tolerance + 1
    return [current_round - tolerance
            + _mix64_int((((seed * GOLDEN) & m) ^ _mix64_int(i + 1)) ^ ROUND_SALT) % span
            for i in range(n)]
