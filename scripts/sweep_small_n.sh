#!/bin/bash
# Few-client shapes (config 1's 10 x 582K MNIST CNN and neighbours): the auto
# fold against the one-block-per-tile, one-wave and lane-per-column variants,
# batched back-to-back launches per variant, shuffled order per round
# (bench.py --sweep).  SHAPES / VARIANTS override the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/small_n}
mkdir -p "$OUT"
SHAPES=${SHAPES:-"10:582026 20:582026 50:582026 10:67267 100:67267 10:1000000"}
VARIANTS=${VARIANTS:-}
for shape in $SHAPES; do
  n=${shape%%:*}; p=${shape##*:}
  echo "== ${n}:${p}"
  timeout -k 10 240 python bench.py --clients "$n" --params "$p" --sweep --variants "$VARIANTS" --steps 10 --warmup 2 \
    --no-cpu-baseline > "$OUT/${n}x${p}.json" 2> "$OUT/${n}x${p}.log" || exit $?
  grep -E "^variant" "$OUT/${n}x${p}.log" | sort -t'>' -k2 -rn | head -8
done
