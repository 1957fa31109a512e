#!/bin/bash
# LDS fold check: the LDS/pointer parity tests, then a narrow-shape variant
# sweep and the pointer-table timings (GPU box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "lds or variant or rowset or narrow or picks or accumulate or ptr or shapes or pitch or chunked or graph" \
  > gpurun_out/colf_tests.log 2>&1 && \
bash scripts/sweep_narrow2.sh ${SHAPES:-1024:16384 1024:67267 256:67267 100:67267 4096:67267 1024:131072} \
  > gpurun_out/colf_sweep.log 2>&1 && \
timeout -k 10 120 python tools/ptrs_bench.py --params 67267 --variants > gpurun_out/colf_ptrs.log 2>&1
