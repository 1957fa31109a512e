#!/bin/bash
# Check at HEAD: the whole GPU suite, smoke(), the default bench line, the C3
# profile (kernel trace + FETCH_SIZE / WRITE_SIZE passes -> pmc_c3.json), and
# 8-rank gloo rehearsals of C3 / C4 with the default slot layouts.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
COMMIT=${COMMIT:-unknown}
exec scripts/gpu_steps.sh \
  "pytest_gpu:600:$PYT -m gpu tests" \
  "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default:300:python3 bench.py" \
  "prof_c3:900:scripts/profile_c3.sh r03 $COMMIT" \
  "rehearse_c3_w8:300:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c3 --clients 16 --steps 2 --warmup 1 --no-cpu-baseline" \
  "rehearse_c4_w8:300:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --clients 32 --steps 2 --warmup 1 --no-cpu-baseline"
