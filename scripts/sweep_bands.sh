#!/bin/bash
# Column-band size of the grid-stride fold (gsband<k>: bands of k passes) by
# client count, plain and stall-aware (C5 is stall-aware 512 x 25M).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/bands}
mkdir -p "$OUT"
for spec in c3:256:40000000 c3:512:20000000 c3:768:13000000 c3:1024:10000000 c5:256:50000000 c5:512:25000000 c5:1024:12500000 c3:128:80000000; do
  IFS=: read -r cfg n p <<< "$spec"
  echo "== $cfg ${n}x${p}"
  timeout -k 10 300 python bench.py --config "$cfg" --clients "$n" --params "$p" --sweep --variants 0,10,13,14,15,12 \
    --steps 8 --warmup 2 --no-cpu-baseline > "$OUT/${cfg}_${n}x${p}.json" 2> "$OUT/${cfg}_${n}x${p}.log" || exit $?
  grep -E "^variant" "$OUT/${cfg}_${n}x${p}.log" | sort -t'>' -k2 -rn
done
