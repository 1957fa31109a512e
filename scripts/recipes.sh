#!/bin/bash
# Named GPU recipes: one parameterised entry point for the gpurun calls of a
# round (replaces the per-check wrapper scripts of rounds 2-3).  Each recipe is
# a list of "name:seconds:command" steps for scripts/gpu_steps.sh (own time
# limit per step, logs in gpurun_out/<name>.log, stops after a timeout/abort).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- scripts/recipes.sh <recipe> [extra steps...]
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
XI="python3 tools/exchange_interference.py"
BF16_DYN="bf16_dyn_u32c1b128,bf16_dyn_u16c1b256,bf16_dyn_u32c1b64,bf16_dyn_u16c2b128,bf16_dyn_u8c2b256,bf16_dyn_u32c1b256"
F32_DYN="gs_bands_16k,dyn_8k,dynp_u32c1b128,dynp_u16c1b256,dynp_u32c1b64,dynp_u16c2b256,dynp_u32c1b256"
recipe=${1:-}
shift || true
case "$recipe" in
  gpu_suite)  # the whole -m gpu suite + smoke
    steps=("pytest_gpu:1100:$T -m gpu tests" "smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'") ;;
  bench)      # the default bench line
    steps=("bench_default:400:python3 bench.py") ;;
  dyn_forms)  # round 4: the dynamic-tile forms, parity and the exchange proxy
    steps=("pytest_shared:700:$T tests/test_gpu_shared_fold.py tests/test_gpu_tuner.py"
           "xi_c4_host:300:$XI --config c4 --host-src --scale 0.15 --forms $BF16_DYN"
           "xi_c4_host_r1:300:$XI --config c4 --host-src --scale 0.15 --forced-rounds overlapped --forms $BF16_DYN"
           "xi_c4_hbm:300:$XI --config c4 --forms $BF16_DYN"
           "xi_c3_host:400:$XI --config c3 --host-src --scale 0.15 --forms $F32_DYN") ;;
  step_forms)  # round 4: the whole step in one launch, parity and the exchange proxy
    S_BF="product,bf16_step_u8c2,bf16_step_u16c2,bf16_step_u8c4,bf16_step_u4c4"
    S_F32="product,f32_step_u8c4,f32_step_u8c2,f32_step_u16c2,f32_step_u16c1"
    steps=("pytest_shared:700:$T tests/test_gpu_shared_fold.py"
           "xi_c4_host_step:300:$XI --config c4 --host-src --scale 0.15 --step-forms $S_BF --forms bf16_bands4_u8c4"
           "xi_c4_hbm_step:300:$XI --config c4 --step-forms $S_BF --forms bf16_bands4_u8c4"
           "xi_c3_host_step:400:$XI --config c3 --host-src --scale 0.15 --step-forms $S_F32 --forms gs_bands_16k"
           "tuner_cold:200:python3 tools/tuner_probe.py --clients 256 --params 3454464 --bf16 --cache gpurun_out/tc.txt"
           "tuner_warm:200:python3 tools/tuner_probe.py --clients 256 --params 3454464 --bf16 --cache gpurun_out/tc.txt"
           "tuner_c3:200:python3 tools/tuner_probe.py --clients 1024 --params 10000000 --cache 0"
           "tuner_vary:200:python3 tools/tuner_probe.py --params 909000 --vary-clients 1000,1024,990,700,1010,512,1000 --cache 0") ;;
  none) steps=() ;;
  *) echo "unknown recipe '$recipe'" >&2; exit 2 ;;
esac
exec scripts/gpu_steps.sh "${steps[@]}" "$@"
