#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
exec scripts/gpu_steps.sh \
  "e2e_trace:400:scripts/e2e_trace.sh" \
  "e2e_multi:300:python3 bench_e2e.py --clients 100 --params 1000000 --reps 10 --no-cpu --devices 0,0 && python3 bench_e2e.py --clients 100 --params 10000000 --reps 5 --no-cpu --devices 0,0"
