#!/bin/bash
# Counter evidence for the bf16 folds (config 4) and C5's traffic:
# per shape N:P (bf16 rows, bench.py --config c4 --params P, one GPU) a kernel
# trace + stats, an SQ pass, then FETCH_SIZE and WRITE_SIZE passes, each its
# own rocprofv3 run; then C5's FETCH / WRITE passes.  Outputs: gpurun_out/bf16/.
#   scripts/gpu_steps.sh "bf16:900:scripts/profile_bf16.sh"
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bf16
SHAPES=${*:-"256:12500000 256:3125000 256:100000000"}
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
for s in $SHAPES; do
    n=${s%%:*}; p=${s##*:}
    tag=n${n}_p${p}
    mkdir -p "$OUT/$tag"
    args="$ROOT/bench.py --config c4 --clients $n --params $p --steps 20 --warmup 3 --no-cpu-baseline"
    echo "== $tag"
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$tag/trace" -o run --output-format csv -- \
        python3 $args > "$OUT/$tag/bench.json" 2> "$OUT/$tag/trace.err"
    timeout -s KILL 180 rocprofv3 --pmc $SQ -d "$OUT/$tag/sq" -o run --output-format csv -- \
        python3 $args > /dev/null 2> "$OUT/$tag/sq.err"
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$tag/fetch" -o run --output-format csv -- \
        python3 $args > /dev/null 2> "$OUT/$tag/fetch.err"
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/$tag/write" -o run --output-format csv -- \
        python3 $args > /dev/null 2> "$OUT/$tag/write.err"
done
mkdir -p "$OUT/c5"
args="$ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5/fetch" -o run --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/c5/fetch.err"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5/write" -o run --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/c5/write.err"
echo done
