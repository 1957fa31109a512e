#!/bin/bash
# Counters for the pointer-table fold vs the stacked fold (1024 x 67K).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ptrsprof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
args="$ROOT/tools/ptrs_bench.py --params 67267 --reps 5"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $args > "$OUT/bench.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $args > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d "$OUT/sq" -o run --output-format csv -- python3 $args > /dev/null
echo done
