#!/bin/bash
# End-to-end (host NPZ blobs -> model) rate over staging-chunk size x slot count,
# alternated twice on one box (FEDAVG_STREAM_CHUNK_MB / FEDAVG_STREAM_SLOTS).
# SHAPES "N:P ...".  Outputs: gpurun_out/e2e_chunks/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/e2e_chunks}
mkdir -p "$OUT"
SHAPES=${SHAPES:-"100:1000000 10:582026 100:10000000"}
CONFIGS=${CONFIGS:-"64:2 32:3 16:4 16:6 8:8 4:12"}
for pass in 1 2; do
  for shape in $SHAPES; do
    n=${shape%%:*}; p=${shape##*:}
    for cfg in $CONFIGS; do
      mb=${cfg%%:*}; sl=${cfg##*:}
      line=$(FEDAVG_STREAM_CHUNK_MB=$mb FEDAVG_STREAM_SLOTS=$sl timeout -k 10 120 python bench_e2e.py --clients $n \
             --params $p --reps 15 --no-cpu 2>>"$OUT/err.log") || exit $?
      echo "$line" >> "$OUT/${n}x${p}_${mb}mb_${sl}slots.jsonl"
      echo "pass $pass ${n}x${p} chunk ${mb}MB slots $sl: $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("gpu_e2e_s"), d.get("gpu_e2e_gbs"))')"
    done
  done
done
