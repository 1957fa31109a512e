#!/bin/bash
# The short-last-round layout and the ingest pipe's abandoned-round drain:
# their GPU tests, then the per-rank fold cost of tail layouts (C4 and C3 ranks).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "tests_tail_pipe:300:$PYT -m gpu tests/test_gpu_rccl.py tests/test_gpu_ingest.py tests/test_gpu_sharding.py" \
  "tail_budget:900:scripts/tail_budget.sh"
