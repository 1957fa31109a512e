#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "shard_tests:300:$PYT -m gpu tests/test_gpu_rccl.py tests/test_gpu_sharding.py" \
  "c4_trace:600:scripts/c4_trace.sh" \
  "c4_budget:600:scripts/c4_budget.sh" \
  "bench_rccl_c3:300:python3 bench.py --rccl-world1 --steps 10"
