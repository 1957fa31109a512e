#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:800:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ptrs:300:for p in 4096 67267 582026; do python tools/ptrs_bench.py --params \$p; done" \
  "small:300:for s in 1024:67267 256:67267 100:67267 1024:16384 1024:4099 100:582026 10:582026; do python bench.py --config c3 --clients \${s%%:*} --params \${s##*:} --steps 200 --warmup 20 --no-cpu-baseline; done" \
  "narrow:900:scripts/profile_narrow.sh 1024:67267 256:67267 1024:16384 10:582026"
