#!/bin/bash
# SQ counters for a few kernel variants on one shape: scripts/profile_variants.sh N P V1,V2,...
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pv_$1_$2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
args="$ROOT/bench.py --config c3 --clients $1 --params $2 --sweep --variants $3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d "$OUT/sq" -o run --output-format csv -- python3 $args > /dev/null 2> "$OUT/sq.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_INSTS_SMEM -d "$OUT/sq2" -o run --output-format csv -- python3 $args > /dev/null 2> "$OUT/sq2.err"
echo done
