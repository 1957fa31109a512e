#!/bin/bash
# Counter evidence for the narrow-model folds, one MI355X:
#   kernel trace + stats, then SQ counters, then FETCH_SIZE, each its own pass,
# for every shape given as N:P (default: speech CNN x1024, MNIST CNN x100,
# config 1's 10 x MNIST CNN, C2).  Outputs under gpurun_out/narrow/.
#   scripts/gpu_steps.sh "narrow:900:scripts/profile_narrow.sh"
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/narrow
SHAPES=${*:-"1024:67267 256:67267 100:582026 10:582026 100:1000000"}
for s in $SHAPES; do mkdir -p "$OUT/n${s%%:*}_p${s##*:}"; done
cd /tmp && export TMPDIR=/tmp
export FEDAVG_AUTOTUNE=0  # the policy form, not a tuned one
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"
for s in $SHAPES; do
    n=${s%%:*}; p=${s##*:}
    tag=n${n}_p${p}
    args="$ROOT/bench.py --config c3 --clients $n --params $p --steps 50 --warmup 5 --no-cpu-baseline"
    echo "== $tag"
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$tag/trace" -o run --output-format csv -- \
        python3 $args > "$OUT/$tag/bench.json" 2> "$OUT/$tag/trace.err"
    timeout -s KILL 120 rocprofv3 --pmc $SQ -d "$OUT/$tag/sq" -o run --output-format csv -- \
        python3 $args > /dev/null 2> "$OUT/$tag/sq.err"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$tag/fetch" -o run --output-format csv -- \
        python3 $args > /dev/null 2> "$OUT/$tag/fetch.err"
done
echo done
