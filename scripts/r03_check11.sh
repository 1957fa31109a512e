#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "ingest_tests:300:$PYT -m gpu tests/test_gpu_ingest.py tests/test_gpu_multigpu.py tests/test_gpu_dropin.py tests/test_properties.py" \
  "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "e2e_trace:400:scripts/e2e_trace.sh" \
  "e2e_lines:600:python3 bench_e2e.py --clients 10 --params 582026 --reps 20 && python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 && python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 && python3 bench_e2e.py --clients 1024 --params 1000000 --reps 5"
