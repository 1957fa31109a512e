#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "even_tests:300:$PYT -m gpu tests/test_gpu_parity.py -k 'even_split or all_variants or every_variant_writes'" \
  "sweep_even:1200:scripts/sweep_even.sh"
