#!/bin/bash
# After the any-alignment folds: the -m gpu suite, smoke, the unaligned sweeps.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "dwsweep:700:bash scripts/sweep_unaligned.sh 1024:16387 100:16387 1024:67267 256:67267 100:67267 1024:131071 1024:582026" \
  "dwptrs:400:for p in 16387 67267 582027; do for n in 100 1024; do python tools/ptrs_bench.py --clients \$n --params \$p | grep clients || exit 1; done; done"
