#!/bin/bash
# After the tuner moved to its own header and took the row-table fold: tuner
# tests, the whole GPU suite, smoke(), the default bench line, and the C3
# profile (trace and counter passes with the tuner off).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
COMMIT=${COMMIT:-unknown}
exec scripts/gpu_steps.sh \
  "tuner_tests:300:FEDAVG_AUTOTUNE_LOG=1 $PYT -m gpu tests/test_gpu_tuner.py" \
  "pytest_gpu:600:$PYT -m gpu tests" \
  "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default:300:python3 bench.py" \
  "prof_c3:900:scripts/profile_c3.sh r03b $COMMIT"
