#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "ingest_tests:300:$PYT -m gpu tests/test_gpu_ingest.py tests/test_gpu_multigpu.py tests/test_gpu_dropin.py" \
  "e2e_ramp:700:OUT=gpurun_out/e2e_ramp CONFIGS='py:64:2 nat:16:4 nat:32:3 nat:64:3' scripts/e2e_native.sh" \
  "c4_budget:600:scripts/c4_budget.sh"
