#!/bin/bash
# The one-wave LDS-DMA narrow fold (k_fold_f32_w1): bit-exactness (every variant,
# every product form), then sweeps of narrow and few-tile shapes against the
# LDS forms, with the tuner's decisions logged.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
NARROW="0,17,20,21,25,41,50,52,53,59,97,106,107,108,109"
exec scripts/gpu_steps.sh \
  "w1_tests:300:$PYT -m gpu tests/test_gpu_tuner.py tests/test_gpu_parity.py -k 'variants or form or tuned'" \
  "grid_narrow:600:OUT=gpurun_out/grid_narrow_w1 VARIANTS=$NARROW NS='100 256 1024 4096' PS='4096 16384 32768 67267 100000 131072 200000' scripts/sweep_even.sh" \
  "grid_few:600:OUT=gpurun_out/grid_few_w1 VARIANTS=0,2,11,17,59,91,94,97,103,106,107 NS='64 100 256 1024' PS='300000 582026 800000' scripts/sweep_even.sh"
