#!/bin/bash
# The tuner with two timed passes in opposite orders: its tests, the probe, the
# mid / narrow grids, the slot shapes, every bench line.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
MID="0,1,2,6,10,11,14,16,17,59,91,92,94,97,103"
NARROW="0,17,20,21,25,41,50,52,53,59,97"
exec scripts/gpu_steps.sh \
  "tuner_tests:300:$PYT -m gpu tests/test_gpu_tuner.py" \
  "probe:300:scripts/r03_probe_tuner.sh" \
  "grid_mid:900:OUT=gpurun_out/grid_mid VARIANTS=$MID scripts/sweep_even.sh" \
  "grid_narrow:600:OUT=gpurun_out/grid_narrow VARIANTS=$NARROW NS='100 256 1024 4096' PS='16384 32768 67267 100000 131072 200000' scripts/sweep_even.sh" \
  "slot_sweep:900:scripts/sweep_bf16_slots.sh" \
  "benches:900:scripts/r03_benches.sh"
