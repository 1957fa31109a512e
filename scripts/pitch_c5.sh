#!/bin/bash
# C5 (512 x 25M fp32 stall-aware) and C3 with extra row padding (bench.py
# --pitch-extra, elements): does the row pitch decide C5's lower fraction of
# its read sweep?  Outputs: gpurun_out/pitch_c5/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/pitch_c5
mkdir -p "$OUT"
for pass in 1 2; do
  for cfg in c5 c3; do
    for pe in 0 64 1024 4096 16384 262144; do
      timeout -k 10 200 python3 bench.py --config $cfg --pitch-extra $pe --steps 10 --warmup 2 --no-cpu-baseline \
        > "$OUT/${cfg}_pe${pe}_p$pass.json" 2> "$OUT/${cfg}_pe${pe}_p$pass.err" || exit $?
      python3 -c "import json; d=json.loads(open('$OUT/${cfg}_pe${pe}_p$pass.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg pitch+$pe pass $pass', r['kernel_ms_avg'], r['achieved'], r['frac_of_read_ceiling'])"
    done
  done
done
