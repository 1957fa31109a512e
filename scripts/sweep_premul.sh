#!/bin/bash
# Premultiplied-stash LDS fold (LOPT bit 3, pm_* variants) against the
# product's LDS picks: variant parity tests, then interleaved sweeps over the
# narrow shapes, plain (c3) and stall-aware (c5).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/premul
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "lds_variants or all_variants or every_variant_writes or any_alignment" > gpurun_out/premul/tests.log 2>&1 || exit 1
tail -3 gpurun_out/premul/tests.log
V=0,17,25,37,41,50,52,53,84,110,111,112,113,114,115,116,117,118
for cfg in c3 c5; do
  for s in 1024:16384 256:16384 4096:16384 1024:4096 1024:67267 256:67267 1024:131072 100:582026; do
    echo "== $cfg $s" | tee -a gpurun_out/premul/sweep.log
    timeout -k 10 120 python bench.py --config $cfg --clients ${s%%:*} --params ${s##*:} --sweep --variants $V \
      --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/premul/one.log 2>&1 || exit 1
    grep -E "variant" gpurun_out/premul/one.log >> gpurun_out/premul/sweep.log
  done
done
