#!/bin/bash
# Row-pitch experiment: the same model size with extra row padding
# (bench.py --pitch-extra, elements), auto fold against the tile / grid-stride
# forms.  SHAPES = N:P list, PADS = extra elements list.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/pitch}
mkdir -p "$OUT"
for shape in ${SHAPES:-1024:800000 100:800000 1024:786000}; do
  n=${shape%%:*}; p=${shape##*:}
  for e in ${PADS:-0 64 128 256 512 1024 2048}; do
    timeout -k 10 200 python bench.py --clients "$n" --params "$p" --pitch-extra "$e" --sweep --variants "${VARIANTS:-0,2,10,11,91}" \
      --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${n}x${p}_e$e.json" 2> "$OUT/${n}x${p}_e$e.log" || exit $?
    echo "${n}x${p} +$e: $(grep -E '^variant' "$OUT/${n}x${p}_e$e.log" | awk '{printf "%s %s | ", $3, $5}')"
  done
done
