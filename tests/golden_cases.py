"""Loader for tests/golden (reference-generated vectors; see golden/make_golden.py)."""
from __future__ import annotations

import json
import os

import numpy as np

from fedlesscan_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

_manifest = None
_arrays = None


def manifest() -> dict:
    global _manifest
    if _manifest is None:
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            _manifest = json.load(f)
    return _manifest


def arrays():
    global _arrays
    if _arrays is None:
        with np.load(os.path.join(GOLDEN, "cases.npz"), allow_pickle=False) as z:
            _arrays = {k: z[k] for k in z.files}
    return _arrays


def _split(row, shapes):
    out, off = [], 0
    for shp in shapes:
        n = int(np.prod(shp)) if len(shp) else 1
        out.append(row[off:off + n].reshape(shp).copy())
        off += n
    return out


def parameters(case: str):
    """Per-client layer lists (List[List[np.ndarray]]) for a golden case."""
    m = manifest()[case]
    A = arrays()
    if m["kind"] == "literal":
        out = []
        for i in range(m["n_clients"]):
            layers = []
            li = 0
            while f"{case}/X/{i}/{li}" in A:
                layers.append(A[f"{case}/X/{i}/{li}"])
                li += 1
            out.append(layers)
        return out
    X = synth.clients_f32(m["seed"], m["n_clients"], 0, m["P"])
    if m["kind"] == "synth_stacked":
        return [[X[i].copy()] for i in range(m["n_clients"])]
    return [_split(X[i], m["shapes"]) for i in range(m["n_clients"])]


def stacked(case: str) -> np.ndarray:
    m = manifest()[case]
    return synth.clients_f32(m["seed"], m.get("n_clients", m.get("rows")), 0, m["P"])


def expected(case: str, prefix: str):
    m = manifest()[case]["outputs"][prefix]
    A = arrays()
    if manifest()[case].get("sampled"):
        return None
    return [A[f"{case}/{prefix}/{li}"] for li in range(m["n_layers"])]


def feats(case: str):
    m = manifest()[case]
    return [{"round_id": r, "client_id": f"c{i}", "session_id": "s"} for i, r in enumerate(m["round_ids"])]


def same_bits(a: np.ndarray, b: np.ndarray, nan_equal: bool = True) -> bool:
    """Bit-for-bit equality; NaNs compare equal regardless of payload/sign
    (x86 numpy yields the negative default NaN, the GPU the positive one)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.dtype.kind != "f":
        return np.array_equal(a, b)
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    ua = a.view(np.uint32 if a.itemsize == 4 else np.uint64)
    ub = b.view(np.uint32 if b.itemsize == 4 else np.uint64)
    return bool(np.array_equal(ua[~na], ub[~nb]))
