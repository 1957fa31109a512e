#!/bin/bash
# Round 3: the even-split fold (k_fold_f32_even) against the product's auto
# pick and the forms the round-2 policy chooses between, over the round-2
# 36-shape grid (profiles/r02_small_n/final/) and the 0.7-0.9 tiles-per-CU band.
# bench.py --sweep: batched back-to-back launches per variant, shuffled order
# per round, medians.  Outputs: gpurun_out/even/<N>x<P>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export FEDAVG_AUTOTUNE_LOG=1  # the tuner's decisions (every candidate's time) go to the stderr logs
OUT=${OUT:-gpurun_out/even}
mkdir -p "$OUT"
NS=${NS:-"10 32 64 80 100 200 1024"}
PS=${PS:-"300000 582026 740000 800000 900000 1000000"}
VARIANTS=${VARIANTS:-"0,1,2,10,11,91,97,98,99,100,101,102,103,104,105"}
for n in $NS; do
  for p in $PS; do
    timeout -k 10 120 python bench.py --clients "$n" --params "$p" --sweep --variants "$VARIANTS" --steps 10 \
      --warmup 2 --no-cpu-baseline > "$OUT/${n}x${p}.json" 2> "$OUT/${n}x${p}.log" || exit $?
    echo "== ${n}x${p}: $(grep -E '^variant' "$OUT/${n}x${p}.log" | sort -t'>' -k2 -rn | head -3 | awk '{print $3, $5}' | tr '\n' ' ')"
  done
done
