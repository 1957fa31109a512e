#!/bin/bash
# 4-byte-load LDS fold: parity on unaligned layouts, then the unaligned sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "dwtests:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'any_alignment or lds_variants or variants_bit or every_variant'" \
  "dwsweep:700:bash scripts/sweep_unaligned.sh"
