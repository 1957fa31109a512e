"""Host-only stress programs of the native pieces, built here with g++ against
simulated HIP runtimes (no GPU): the tuner's state machine (tools/tuner_stress.cpp,
fedlesscan_amd/csrc/tuner.hpp) and the native ingest pipe
(tools/ingest_pipe_stress.cpp, csrc/ingest_pipe.cpp).  The sanitizer builds
are tools/tuner_stress.sh and tools/ingest_pipe_stress.sh."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_and_run(tmp_path, name, srcs, inc):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O1", *[f"-I{os.path.join(REPO, i)}" for i in inc], "-o", exe,
           *[os.path.join(REPO, s) for s in srcs], "-pthread"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_tuner_state_machine(tmp_path):
    out = _build_and_run(tmp_path, "tuner_stress", ["tools/tuner_stress.cpp"],
                         ["tools/tunersim", "fedlesscan_amd/csrc"])
    assert "tuner_stress: ok" in out


def test_ingest_pipe_host_stress(tmp_path):
    out = _build_and_run(tmp_path, "ingest_pipe_stress",
                         ["tools/ingest_pipe_stress.cpp", "fedlesscan_amd/csrc/ingest_pipe.cpp"],
                         ["tools/hipsim", "include", "fedlesscan_amd/csrc"])
    assert "ingest_pipe_stress: ok" in out
