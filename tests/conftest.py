import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)
# The library's tuner persists its decisions (FEDAVG_TUNE_CACHE); tests start
# from an empty cache of their own so that they see every shape measured.
if "FEDAVG_TUNE_CACHE" not in os.environ:
    import tempfile
    os.environ["FEDAVG_TUNE_CACHE"] = os.path.join(tempfile.mkdtemp(prefix="fa_tune_test_"), "tuner.txt")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # A gpu-marked test on a machine without a GPU is an error only when the
    # user explicitly selected gpu tests; otherwise it is skipped.
    if _gpu_available():
        return
    markexpr = config.getoption("-m") or ""
    if "gpu" in markexpr and "not gpu" not in markexpr:
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
