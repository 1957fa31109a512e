#!/bin/bash
# Any-alignment pointer folds: parity, then timings on unaligned row tables.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "dwtests:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'ptrs or any_alignment or rowset'" \
  "dwptrs:400:for p in 16387 67267 582027 2500001; do for n in 100 1024; do python tools/ptrs_bench.py --clients \$n --params \$p --variants | grep clients || exit 1; done; done"
