#!/bin/bash
# After the narrow pick moved to the premultiplied stash (LOPT 8, 6 chunks):
# the auto fold against the previous form (lds4_w2r32t16) on the narrow shapes,
# plain and stall-aware, then the kernel trace + counters of the narrow shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/premul2
for cfg in c3 c5; do
  for s in 1024:16384 256:16384 4096:16384 1024:4096 1024:32768 64:16384 1024:30000; do
    echo "== $cfg $s" >> gpurun_out/premul2/sweep.log
    timeout -k 10 120 python bench.py --config $cfg --clients ${s%%:*} --params ${s##*:} --sweep --variants 0,41,117,110 \
      --steps 30 --warmup 2 --no-cpu-baseline > gpurun_out/premul2/one.log 2>&1 || exit 1
    grep -E "variant" gpurun_out/premul2/one.log >> gpurun_out/premul2/sweep.log
  done
done
echo sweep done
bash scripts/profile_narrow.sh 1024:16384 256:16384 4096:16384
