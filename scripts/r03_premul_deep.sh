#!/bin/bash
# Deeper / longer-chunk forms of the premultiplied narrow fold (pm_lds8/10, r64).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/premul4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "lds_variants or all_variants or every_variant_writes" > gpurun_out/premul4/tests.log 2>&1 || exit 1
tail -1 gpurun_out/premul4/tests.log
for cfg in c3 c5; do
  for s in 1024:16384 4096:16384 256:16384 1024:4096 1024:32768 1024:24000 64:16384; do
    echo "== $cfg $s" >> gpurun_out/premul4/sweep.log
    timeout -k 10 120 python bench.py --config $cfg --clients ${s%%:*} --params ${s##*:} --sweep \
      --variants 0,110,117,123,124,125,126 --steps 30 --warmup 2 --no-cpu-baseline > gpurun_out/premul4/one.log 2>&1 || exit 1
    grep -E "^variant" gpurun_out/premul4/one.log >> gpurun_out/premul4/sweep.log
  done
done
