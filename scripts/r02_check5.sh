#!/bin/bash
# After the LDS fold changes (column fold, two-wave narrow pick, pointer
# ring): the -m gpu suite, smoke, the narrow-shape sweep and pointer variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "sweep:500:bash scripts/sweep_narrow2.sh 1024:16384 256:16384 4096:16384 1024:30000 1024:67267 100:67267 1024:131072" \
  "ptrs:300:bash scripts/ptrs_variants.sh"
