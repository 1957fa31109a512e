#!/bin/bash
# The fold stream leaving 16 CUs to the collective (CU mask) against the
# exchange proxy: copy unmasked (as RCCL's kernels) or on exactly the free CUs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
X="timeout -k 10 300 python3 tools/exchange_interference.py --host-src --scale 0.15"
OUT=gpurun_out/cumask
mkdir -p $OUT
$X --config c3 --forms gs_bands_16k,dyn_8k --blocks 16,64 > $OUT/c3_all.log 2>&1 &&
$X --config c3 --fold-free 16 --forms gs_bands_16k,dyn_8k --blocks 16,64 > $OUT/c3_free16.log 2>&1 &&
$X --config c3 --fold-free 16 --copy-on-free --forms gs_bands_16k,dyn_8k --blocks 16,64 > $OUT/c3_free16_placed.log 2>&1 &&
$X --config c4 --fold-free 16 --blocks 16,64 > $OUT/c4_free16.log 2>&1 &&
$X --config c4 --fold-free 16 --copy-on-free --blocks 16,64 > $OUT/c4_free16_placed.log 2>&1
