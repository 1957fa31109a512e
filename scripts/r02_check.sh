#!/bin/bash
# Round-2 GPU check: the -m gpu suite, smoke, the pointer-list timings, the
# default bench, and a 2-rank rehearsal of the multi-GPU bench path (both
# ranks on the one GPU, gather through gloo: throughput meaningless).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
scripts/gpu_steps.sh \
  "pytest:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "ptrs:300:for p in 67267 1000000 10000000; do python tools/ptrs_bench.py --params \$p; done" \
  "bench:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "rehearse_c4:400:FEDAVG_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config c4 --steps 3 --warmup 1" \
  "rehearse_c3:400:FEDAVG_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c3 --clients 256 --steps 3 --warmup 1"
