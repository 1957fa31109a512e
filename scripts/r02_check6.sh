#!/bin/bash
# Host-factor entries: the -m gpu suite, smoke, host overhead and pointer timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "host:200:python tools/host_overhead.py" \
  "ptrs:300:for p in 16384 67267 1000000; do python tools/ptrs_bench.py --params \$p; done"
