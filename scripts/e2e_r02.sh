#!/bin/bash
# End-to-end (host NPZ blobs -> GPU result) table of DESIGN.md section 7, plus the
# phase breakdown of the small cases.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "e2e:900:python bench_e2e.py --clients 10 --params 582026 --reps 20 && python bench_e2e.py --clients 100 --params 1000000 --reps 10 && python bench_e2e.py --clients 1024 --params 1000000 --reps 5 && python bench_e2e.py --clients 100 --params 10000000 --reps 5 && python bench_e2e.py --clients 100 --params 10000000 --reps 5 --bson" \
  "phases:600:python tools/e2e_phases.py --clients 10 --params 582026 --reps 10 && python tools/e2e_phases.py --clients 100 --params 1000000 --reps 5"
