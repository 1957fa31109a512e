#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "gpu_suite:900:$PYT -m gpu tests" \
  "c4_trace:600:scripts/c4_trace.sh" \
  "e2e_lines:600:python3 bench_e2e.py --clients 10 --params 582026 --reps 20 && python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 && python3 bench_e2e.py --clients 100 --params 10000000 --reps 5 && python3 bench_e2e.py --clients 100 --params 10000000 --reps 5 --bson && python3 bench_e2e.py --clients 1024 --params 1000000 --reps 5" \
  "bench_default:300:python3 bench.py"
