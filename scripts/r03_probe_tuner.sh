#!/bin/bash
# What the tuner measures on the shapes where it chose wrong (grid_mid: 100 x 300K
# took gs_bands_16k, 1.79x the lane-per-column form), isolated vs back-to-back calls.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export FEDAVG_AUTOTUNE_LOG=1
for shape in "100 300000" "64 582026" "100 582026" "1024 909120" "100 1000000"; do
  set -- $shape
  timeout -k 10 60 python3 tools/tuner_probe.py --clients $1 --params $2 || exit $?
  timeout -k 10 60 python3 tools/tuner_probe.py --clients $1 --params $2 --b2b || exit $?
done
