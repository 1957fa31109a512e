#!/bin/bash
# Pointer-table fold: loader/tile variants, kernel alone, per model width (GPU box).
set -o pipefail
mkdir -p gpurun_out
for p in ${PARAMS:-16384 67267 131072 200001 30000}; do
  timeout -k 10 120 python tools/ptrs_bench.py --params $p --clients ${CLIENTS:-1024} --variants 2>&1 | grep clients || exit 1
done
