#!/bin/bash
# Counter evidence for one 8-GPU C3 rank's step on one GPU (round 5): 1024
# clients x the rank's four fp32 slots (sharding.overlap_layout, 10M columns)
# through tools/exchange_interference.py with no copy: the one-launch step
# (k_fold_f32_step, write-through tile stores) and the per-round policy
# launches, tuner off.  A kernel trace, FETCH_SIZE and WRITE_SIZE passes (each
# its own rocprofv3 run), then profiles-ready summaries.
#   scripts/gpu_steps.sh "prof_c3r:900:scripts/profile_c3_rank.sh <tag> <commit>"
set -euo pipefail
TAG=${1:-r05}
COMMIT=${2:-unknown}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_c3r_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export FEDAVG_AUTOTUNE=0
STEPS=6
args="$ROOT/tools/exchange_interference.py --config c3 --blocks '' --steps $STEPS --step-forms product"
eval timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o c3r --output-format csv -- \
    python3 $args > "$OUT/trace.log" 2> "$OUT/trace.err"
eval timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o c3r --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/fetch.err"
eval timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o c3r --output-format csv -- \
    python3 $args > /dev/null 2> "$OUT/write.err"
cd "$ROOT"
# the rank's algorithmic bytes: 1024 x 10M x 4 read + 10M x 4 written
python3 scripts/pmc_traffic.py --fetch "$OUT/fetch" --write "$OUT/write" \
    --kernel "k_fold_f32_step<8, 4, 16, 1" --bytes 41000000000 \
    --provenance "rocprofv3 passes of tools/exchange_interference.py --config c3 (no copy), round $TAG, commit $COMMIT, $(date -u +%Y-%m-%dT%H:%MZ)" \
    --out "$OUT/pmc_c3_rank_step.json"
echo done
