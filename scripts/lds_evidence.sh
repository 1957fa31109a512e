#!/bin/bash
# Reproduces profiles/r02_lds/ (the LDS-fold work of late round 2) on one MI355X:
# the LDS / pointer / alignment parity tests, the narrow-shape variant sweeps
# (loader and fold A/B: o<LOPT>_*, qf_* variants), the small-P sweep, the
# unaligned-row sweep, pointer-table variants and timings, and the host cost
# per call.  Outputs in gpurun_out/ (one log per step).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "lds_tests:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'lds or variant or rowset or ptrs or any_alignment or host_factor'" \
  "loader_ab_sweep:500:bash scripts/sweep_narrow2.sh 1024:16384 1024:67267 256:67267 100:67267 4096:67267 1024:131072" \
  "sweep_small:500:bash scripts/sweep_narrow2.sh 1024:16384 256:16384 100:16384 4096:16384 1024:4096 1024:30000 10:16384" \
  "dw_sweep:700:bash scripts/sweep_unaligned.sh" \
  "ptrs_variants:400:bash scripts/ptrs_variants.sh" \
  "ptrs_large:400:for p in 1000000 4000000 10000000; do for n in 100 1024; do python tools/ptrs_bench.py --clients \$n --params \$p --variants --reps 10 | grep clients || exit 1; done; done" \
  "host_overhead:200:python tools/host_overhead.py && python tools/host_overhead.py --params 16384"
