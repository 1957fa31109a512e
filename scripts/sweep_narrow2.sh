#!/bin/bash
# Variant sweep (interleaved, shuffled order per round) over narrow shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
SHAPES=${*:-"1024:16384 1024:67267 256:67267 100:67267 4096:67267 1024:582026 100:582026 1024:1000000"}
for s in $SHAPES; do
  echo "== $s"
  timeout -k 10 120 python bench.py --config c3 --clients ${s%%:*} --params ${s##*:} --sweep --steps 20 --warmup 2 --no-cpu-baseline 2>&1 | grep -E "variant|value" | sort -t'>' -k2 -g | tail -50 || exit 1
done
