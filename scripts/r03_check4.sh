#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "native_tests:300:$PYT -m gpu tests/test_gpu_ingest.py tests/test_gpu_multigpu.py tests/test_gpu_dropin.py tests/test_handler_golden.py" \
  "gpu_suite:900:$PYT -m gpu tests" \
  "e2e_native:1000:scripts/e2e_native.sh"
