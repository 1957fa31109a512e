#!/bin/bash
# Round-3 check at HEAD after the container restore: the whole GPU suite,
# smoke(), the default bench line, and 8-rank gloo rehearsals (ranks share
# the box's one GPU: checks the world-8 layout and gather, not throughput).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "pytest_gpu:600:$PYT -m gpu tests" \
  "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default:300:python3 bench.py" \
  "rehearse_c3_w8:300:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c3 --clients 16 --steps 2 --warmup 1 --no-cpu-baseline" \
  "rehearse_c4_w8:300:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --clients 32 --steps 2 --warmup 1 --no-cpu-baseline"
