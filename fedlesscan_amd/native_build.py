"""Build the native libraries in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m fedlesscan_amd.native_build [--force] [--isa]

  libfedavg_hip.so        the product: fedavg.hip (+ fold_kernels.hpp) and the
                          host ingest (NPZ index / pack, BSON walk)
  libfedavg_hip_bench.so  bench / tuning support: fedavg_bench.hip (kernel
                          variants, HBM input generator, read-sweep calibration)
  _hostfast.<abi>.so      host-only CPython helper (gcc): rounding a list of
                          Python weights to float32 in one C loop (hostfast.c)

All compile in parallel.  The .so files land in fedlesscan_amd/_native/
(git-ignored, but shipped to the GPU box by gpurun with the rest of the tree).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SRC = os.path.join(CSRC, "fedavg.hip")
BENCH_SRC = os.path.join(CSRC, "fedavg_bench.hip")
KERNELS = os.path.join(CSRC, "fold_kernels.hpp")
TUNER = os.path.join(CSRC, "tuner.hpp")
HOST_SRCS = [os.path.join(CSRC, f) for f in ("ingest_host.cpp", "bson_host.cpp", "ingest_pipe.cpp")]
HDR = os.path.join(REPO, "include", "fedavg_hip.h")
BENCH_HDR = os.path.join(REPO, "include", "fedavg_hip_bench.h")
OUT_DIR = os.path.join(PKG, "_native")
LIB = os.path.join(OUT_DIR, "libfedavg_hip.so")
BENCH_LIB = os.path.join(OUT_DIR, "libfedavg_hip_bench.so")
HOSTFAST_SRC = os.path.join(CSRC, "hostfast.c")
HOSTFAST = os.path.join(OUT_DIR, "_hostfast" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))  # = _lib.HOSTFAST_PATH
# library -> (sources compiled into it, files it depends on)
TARGETS = {
    LIB: ([SRC, *HOST_SRCS], [SRC, KERNELS, TUNER, HDR, *HOST_SRCS, os.path.join(CSRC, "host_copy.hpp"),
                              os.path.join(CSRC, "peer_exchange.hpp")]),
    BENCH_LIB: ([BENCH_SRC], [BENCH_SRC, KERNELS, TUNER, HDR, BENCH_HDR]),
    HOSTFAST: ([HOSTFAST_SRC], [HOSTFAST_SRC]),
}
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


def _stale(lib: str) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in TARGETS[lib][1])


def build(force: bool = False, isa_dir: str | None = None) -> str:
    """Compile every stale library (all of them with force); returns the product path."""
    os.makedirs(OUT_DIR, exist_ok=True)
    jobs = []
    for lib, (srcs, _) in TARGETS.items():
        if not force and not _stale(lib):
            continue
        tmp = lib + ".tmp"
        cwd = None
        if lib == HOSTFAST:
            cc = os.environ.get("CC") or shutil.which("gcc") or "cc"
            cmd = [cc, "-O2", "-shared", "-fPIC", "-Wall", "-I", sysconfig.get_paths()["include"], "-o", tmp, *srcs]
            jobs.append((lib, tmp, subprocess.Popen(cmd)))
            continue
        cmd = [hipcc(), *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), "-o", tmp, *srcs]
        if isa_dir:
            cwd = os.path.join(isa_dir, os.path.basename(lib).split(".")[0])
            os.makedirs(cwd, exist_ok=True)
            cmd.insert(1, "-save-temps")
        jobs.append((lib, tmp, subprocess.Popen(cmd, cwd=cwd)))
    failed = [lib for lib, _, p in jobs if p.wait() != 0]
    # the HIP libraries are installed even when only the optional CPython
    # helper failed (e.g. a host without Python headers): engine then takes its
    # numpy path for the factor rounding, which gives the same bits
    for lib, tmp, _ in jobs:
        if lib not in failed:
            os.replace(tmp, lib)
    if HOSTFAST in failed:
        print(f"warning: optional helper {os.path.basename(HOSTFAST)} failed to build; "
              "engine rounds the weights with numpy instead", file=sys.stderr)
        failed.remove(HOSTFAST)
    if failed:
        raise RuntimeError(f"native build failed for {', '.join(os.path.basename(f) for f in failed)}")
    return LIB


if __name__ == "__main__":
    force = "--force" in sys.argv
    isa = os.path.join(REPO, "build", "isa") if "--isa" in sys.argv else None
    print(build(force=force, isa_dir=isa))
