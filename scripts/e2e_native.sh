#!/bin/bash
# End-to-end rate with the native ingest pipe over chunk size x slots, against
# the round-2 Python pipeline (FEDAVG_NATIVE_INGEST=0, 64 MB x 2), alternated
# three times on one box.  Outputs: gpurun_out/e2e_native/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/e2e_native}
mkdir -p "$OUT"
SHAPES=${SHAPES:-"100:1000000 10:582026 100:10000000 1024:1000000"}
CONFIGS=${CONFIGS:-"py:64:2 nat:8:4 nat:16:4 nat:16:6 nat:32:3 nat:32:4 nat:64:3"}
for pass in 1 2 3; do
  for shape in $SHAPES; do
    n=${shape%%:*}; p=${shape##*:}
    for cfg in $CONFIGS; do
      kind=${cfg%%:*}; rest=${cfg#*:}; mb=${rest%%:*}; sl=${rest##*:}
      nat=1; [ "$kind" = py ] && nat=0
      line=$(FEDAVG_NATIVE_INGEST=$nat FEDAVG_STREAM_CHUNK_MB=$mb FEDAVG_STREAM_SLOTS=$sl timeout -k 10 150 \
             python bench_e2e.py --clients $n --params $p --reps 15 --no-cpu 2>>"$OUT/err.log") || exit $?
      echo "$line" >> "$OUT/${n}x${p}_${kind}_${mb}mb_${sl}.jsonl"
      echo "pass $pass ${n}x${p} $kind ${mb}MB x$sl: $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["gpu_e2e_s"], d["gpu_e2e_min_s"], d["gpu_e2e_gbs"], d["h2d_pinned_gbs"])')"
    done
  done
done
