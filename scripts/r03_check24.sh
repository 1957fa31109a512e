#!/bin/bash
# Dynamic-tile fold: every form bit-exact (tuner tests), then the exchange
# interference proxy with static and dynamic forms.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "tuner_tests:300:$PYT -m gpu tests/test_gpu_tuner.py" \
  "xi_c3:400:python3 tools/exchange_interference.py --config c3 --forms gs_bands_16k,dyn_16k,dyn_8k,gs_bal_8k,tile_16k_ps --blocks 16,64" \
  "xi_c4:300:python3 tools/exchange_interference.py --config c4 --blocks 16,64"
