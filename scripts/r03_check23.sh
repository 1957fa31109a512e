#!/bin/bash
# HEAD check: the whole GPU suite, smoke(), the default bench line.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "pytest_gpu:600:$PYT -m gpu tests" \
  "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default:300:python3 bench.py"
