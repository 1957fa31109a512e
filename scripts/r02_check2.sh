#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:700:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'ptr or rowset or view_rows'" \
  "ptrs:300:for p in 4096 67267 582026 1000000; do python tools/ptrs_bench.py --params \$p; done" \
  "narrow:900:scripts/profile_narrow.sh"
