#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "pick_tests:300:$PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_ingest.py tests/test_gpu_multigpu.py" \
  "sweep_even2:900:OUT=gpurun_out/even2 VARIANTS=0,1,2,10,11,91,97 scripts/sweep_even.sh" \
  "e2e_chunks:1100:scripts/e2e_chunks.sh"
