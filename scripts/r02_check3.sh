#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "ptrs:300:for p in 67267 1000000; do python tools/ptrs_bench.py --params \$p; done" \
  "host:300:python tools/host_overhead.py && python tools/host_overhead.py --clients 100 --params 1000000" \
  "bench_c2:300:python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline" \
  "bench_small:300:python bench.py --config c3 --clients 1024 --params 67267 --steps 200 --warmup 20 --no-cpu-baseline"
