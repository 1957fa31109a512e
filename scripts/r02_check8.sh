#!/bin/bash
# After the pointer-fold picks: the -m gpu suite, smoke, pointer timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "ptrs:400:for p in 67267 582027 1000000 2500001 4000000; do for n in 100 1024; do python tools/ptrs_bench.py --clients \$n --params \$p --reps 10 | grep clients || exit 1; done; done"
