#!/bin/bash
# round 5 ad-hoc measurements (scripts/gpu_steps.sh steps); see DESIGN.md for what each answered
XI="python3 tools/exchange_interference.py"
FB="python3 tools/bf16_forms_bench.py --clients 256"
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
NOACQ=bf16_step_rt_u8c4n8c2_p100_last_noacq
exec scripts/gpu_steps.sh \
 "pytest_sharding:600:$T tests/test_gpu_sharding.py tests/test_gpu_shared_fold.py tests/test_gpu_rccl.py" \
 "xi_acq:300:$XI --config c4 --blocks '' --steps 30 --step-forms product,$NOACQ,product,$NOACQ" \
 "fb_bucket2x:300:$FB --params 12500000 --forms bf16_bands4_u8c2,bf16_bands4x2_u8c4,bf16_bands4x2_u8c2,bf16_bands4x2_u4c4,bf16_bands4_u8c2" \
 "fb_slot0_2x:300:$FB --params 4934912 --forms bf16_bands4_u8c4,bf16_bands4x2_u8c4,bf16_bands4x2_u8c2,bf16_bands4x2_u4c4,bf16_bands4_u8c4" \
 "prof_c4:600:scripts/profile_c4_rank.sh r05 ${COMMIT:-wip}" \
 "pack_g32:300:python3 tools/pack_bw.py --buckets 1,2,4,8 --rows 32 --threads-per-bucket 32" \
 "rehearse_peer_w8:600:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --steps 2 --warmup 1 --no-cpu-baseline --step-mode one --exchange peer_copy"
