#!/bin/bash
# Rows that are not 16-B aligned (row pitch = an odd model size): the product
# fold against the 4-byte-load LDS variants and the scalar fold (GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
SHAPES=${*:-"1024:16387 1024:67267 100:67267 100:582026 1024:582026 100:1000003 1024:2500001 1024:10000001"}
V=0,84,85,86,87,88,89,90,91
for s in $SHAPES; do
  echo "== $s"
  timeout -k 10 200 python bench.py --config c3 --clients ${s%%:*} --params ${s##*:} --unpadded --sweep \
    --variants $V --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep -E "variant" | sort -t'>' -k2 -g || exit 1
done
