#!/bin/bash
# Counter evidence for one 8-GPU C4 rank's step on one GPU:
# 256 clients x the rank's four bf16 slots (sharding.overlap_layout(100M, 8,
# "bf16"), 12.5M columns; the RNE-bf16 result only, ABI 5: 6.425 GB per step)
# through tools/exchange_interference.py with no copy:
# the product's one-launch step (k_fedavg_bf16_step) and the per-round policy
# launches (k_fedavg_bf16_gs band forms), tuner off.  A kernel trace + stats,
# an SQ pass, FETCH_SIZE and WRITE_SIZE passes (each its own rocprofv3 run),
# then profiles-ready summaries.  Outputs: gpurun_out/prof_c4_<tag>/.
#   scripts/gpu_steps.sh "prof_c4:900:scripts/profile_c4_rank.sh <tag> <commit> [step forms]"
set -euo pipefail
TAG=${1:-r05}
COMMIT=${2:-unknown}
FORMS=${3:-product}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_c4_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export FEDAVG_AUTOTUNE=0
STEPS=10
args="$ROOT/tools/exchange_interference.py --config c4 --blocks '' --steps $STEPS --step-forms $FORMS"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
eval timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o c4 --output-format csv -- \
    python3 $args > "$OUT/trace.log" 2> "$OUT/trace.err"
eval timeout -s KILL 240 rocprofv3 --pmc $SQ -d "$OUT/sq" -o c4 --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/sq.err"
eval timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o c4 --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/fetch.err"
eval timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o c4 --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/write.err"
cd "$ROOT"
# the one-launch step: one dispatch per step (3 warm-up + STEPS timed per step form)
python3 scripts/pmc_traffic.py --fetch "$OUT/fetch" --write "$OUT/write" --sq "$OUT/sq" \
    --kernel "k_fedavg_bf16_step<8, 4, 8, 2" --bytes 6425000000 \
    --provenance "rocprofv3 passes of tools/exchange_interference.py --config c4 (no copy), round $TAG, commit $COMMIT, $(date -u +%Y-%m-%dT%H:%MZ)" \
    --out "$OUT/pmc_c4_rank_step.json"
# the per-round policy launches: 3 + 2 warm-up + STEPS timed steps, several band dispatches each
python3 scripts/pmc_traffic.py --fetch "$OUT/fetch" --write "$OUT/write" --sq "$OUT/sq" \
    --kernel "k_fedavg_bf16_gs" --bytes 6425000000 --calls $((5 + STEPS)) \
    --provenance "rocprofv3 passes of tools/exchange_interference.py --config c4 (no copy), round $TAG, commit $COMMIT, $(date -u +%Y-%m-%dT%H:%MZ)" \
    --out "$OUT/pmc_c4_rank_perround.json"
echo done
