#!/bin/bash
# With the tuner: every bench line; the 42-shape mid-band grid (round-3 grid of
# sweep_even.sh) and a narrow grid, the tuned auto fold against the policy's
# forms and the tuner's candidates.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
MID="0,1,2,6,10,11,14,16,17,59,91,92,94,97,103"
NARROW="0,17,20,21,25,41,50,52,53,59,97"
exec scripts/gpu_steps.sh \
  "benches:900:scripts/r03_benches.sh" \
  "grid_mid:900:OUT=gpurun_out/grid_mid VARIANTS=$MID scripts/sweep_even.sh" \
  "grid_narrow:600:OUT=gpurun_out/grid_narrow VARIANTS=$NARROW NS='100 256 1024 4096' PS='16384 32768 67267 100000 131072 200000' scripts/sweep_even.sh"
