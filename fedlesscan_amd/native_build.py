"""Build libfedavg_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m fedlesscan_amd.native_build [--force] [--isa]

The .so lands in fedlesscan_amd/_native/ (git-ignored, but shipped to the GPU
box by gpurun with the rest of the tree).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "fedavg.hip")
HOST_SRCS = [os.path.join(PKG, "csrc", f) for f in ("ingest_host.cpp", "bson_host.cpp")]
HDR = os.path.join(REPO, "include", "fedavg_hip.h")
OUT_DIR = os.path.join(PKG, "_native")
LIB = os.path.join(OUT_DIR, "libfedavg_hip.so")
ARCH = os.environ.get("FEDAVG_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: multiply and add must stay separate (numpy semantics);
# no -ffast-math / denormal flushing: IEEE divide and subnormals as numpy.
HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
               f"--offload-arch={ARCH}", "-Wall"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in (SRC, *HOST_SRCS, HDR))


def build(force: bool = False, isa_dir: str | None = None) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), "-o", tmp, SRC, *HOST_SRCS]
    if isa_dir:
        os.makedirs(isa_dir, exist_ok=True)
        cmd.insert(1, "-save-temps")
        subprocess.check_call(cmd, cwd=isa_dir)
    else:
        subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    force = "--force" in sys.argv
    isa = os.path.join(REPO, "build", "isa") if "--isa" in sys.argv else None
    print(build(force=force, isa_dir=isa))
