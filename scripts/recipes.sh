#!/bin/bash
# Named GPU recipes: the one parameterised entry point for gpurun calls (it
# replaces the per-check wrapper scripts of rounds 2-3).  Each recipe is a list
# of "name:seconds:command" steps for scripts/gpu_steps.sh: each step has its
# own time limit, logs to gpurun_out/<name>.log, and a timeout / abort / fault
# stops the call.  Extra steps may follow the recipe name.
#   /usr/local/graft/bin/gpurun --timeout 1500 -- scripts/recipes.sh <recipe> ["name:secs:cmd" ...]
# Recipes:
#   gpu_suite     the whole -m gpu suite + smoke (the driver's round-end checks)
#   bench         the default bench line (C3, the headline)
#   bench_lines   every BASELINE bench line (scripts/bench_lines.sh)
#   prof_c3       C3 bench line + kernel trace + FETCH/WRITE_SIZE passes (scripts/profile_c3.sh TAG COMMIT)
#   rehearse_w8   8 ranks sharing the one GPU over gloo: C3 weak and C4 strong (the driver's 8-GPU recipe
#                 is `python bench.py --gpus 8` and `python bench.py --gpus 8 --config c4`)
#   c4_rank       one 8-GPU C4 rank on one GPU under nccl at world 1: one launch per step vs per round
#   exchange      the exchange-interference proxy (tools/exchange_interference.py), C4 and C3 ranks
#   exchange_sdma the same proxy with copy-engine copies (hipMemcpyAsync, no CUs) beside the fold
#   changed       the GPU tests of round 5's changes (step forms, sharding, RCCL world 1, tuner, host)
#   e2e           end-to-end from host NPZ blobs: config-1 shapes, C2, 1024 x 1M, and C3 (1024 x 10M)
#   tuner         the tuner's first-call cost, cold and with a warm cache file; varying client counts
#   final         gpu_suite + bench + prof_c3 (the end-of-round evidence)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
XI="python3 tools/exchange_interference.py"
TAG=${TAG:-r05}
COMMIT=${COMMIT:-unknown}
S_BF="product,bf16_step_rt_u8c4n8c2_p100_last,bf16_step_static_u8c4"
S_F32="product"
C4R="--config c4 --params 12500000 --rounds 4 --steps 30 --warmup 5 --no-cpu-baseline"
recipe=${1:-}
shift || true
case "$recipe" in
  gpu_suite)
    steps=("pytest_gpu:1100:$T -m gpu tests" "smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'") ;;
  bench)
    steps=("bench_default:500:python3 bench.py") ;;
  bench_lines)
    steps=("bench_lines:1100:scripts/bench_lines.sh") ;;
  prof_c3)
    steps=("prof_c3:900:scripts/profile_c3.sh $TAG $COMMIT") ;;
  rehearse_w8)
    steps=("rehearse_c3_w8:400:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c3 --clients 16 --steps 2 --warmup 1 --no-cpu-baseline"
           "rehearse_c4_w8:600:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --steps 2 --warmup 1 --no-cpu-baseline"
           "rehearse_c4_w8_perround:600:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --steps 2 --warmup 1 --no-cpu-baseline --per-round-launches"
           "rehearse_peer_w8:600:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --steps 3 --warmup 1 --no-cpu-baseline --exchange peer_copy --step-mode one"
           "rehearse_c4_w8_loop:600:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --config c4 --steps 2 --warmup 1 --no-cpu-baseline --step-impl loop") ;;
  c4_rank)
    steps=("c4_rank_one:300:python3 bench.py --rccl-world1 $C4R --step-mode one"
           "c4_rank_perround:300:python3 bench.py --rccl-world1 $C4R --per-round-launches"
           "c3_rank_one:300:python3 bench.py --rccl-world1 --config c3 --rounds 4 --steps 10 --no-cpu-baseline --step-mode one"
           "c3_rank_perround:300:python3 bench.py --rccl-world1 --config c3 --rounds 4 --steps 10 --no-cpu-baseline --per-round-launches") ;;
  exchange)
    steps=("xi_c4_host:300:$XI --config c4 --host-src --scale 0.15 --step-forms $S_BF"
           "xi_c4_hbm:300:$XI --config c4 --step-forms $S_BF"
           "xi_c3_host:400:$XI --config c3 --host-src --scale 0.15 --step-forms $S_F32") ;;
  exchange_sdma)  # round 5: the fold beside copy-engine traffic
    steps=("xsd_c4_full:300:$XI --config c4 --copy sdma --blocks 1 --step-forms product"
           "xsd_c4_015:300:$XI --config c4 --copy sdma --scale 0.15 --blocks 1 --step-forms product"
           "xsd_c3_full:400:$XI --config c3 --copy sdma --blocks 1 --step-forms product"
           "xk_c4_host:300:$XI --config c4 --host-src --scale 0.15 --step-forms product") ;;
  changed)
    steps=("pytest_changed:900:$T tests/test_gpu_shared_fold.py tests/test_gpu_sharding.py tests/test_gpu_rccl.py tests/test_gpu_tuner.py tests/test_host.py") ;;
  e2e)
    steps=("e2e_small:600:python3 bench_e2e.py --clients 10 --params 582026 --reps 20 && python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 && python3 bench_e2e.py --clients 1024 --params 1000000 --reps 5"
           "e2e_c3:900:python3 bench_e2e.py --clients 1024 --params 10000000 --reps 3 --no-cpu --check-cols 1000000") ;;
  tuner)
    steps=("tuner_cold:200:python3 tools/tuner_probe.py --clients 256 --params 3454464 --bf16 --cache gpurun_out/tc.txt"
           "tuner_warm:200:python3 tools/tuner_probe.py --clients 256 --params 3454464 --bf16 --cache gpurun_out/tc.txt"
           "tuner_c3:200:python3 tools/tuner_probe.py --clients 1024 --params 10000000 --cache 0"
           "tuner_vary:200:python3 tools/tuner_probe.py --params 909000 --vary-clients 1000,1024,990,700,1010,512,1000 --cache 0") ;;
  step_forms)  # round 4: the one-launch step, its parity and the proxy
    steps=("pytest_shared:700:$T tests/test_gpu_shared_fold.py tests/test_gpu_sharding.py tests/test_gpu_rccl.py"
           "xi_c4_host_step:300:$XI --config c4 --host-src --scale 0.15 --step-forms $S_BF"
           "xi_c4_hbm_step:300:$XI --config c4 --step-forms $S_BF"
           "xi_c3_host_step:400:$XI --config c3 --host-src --scale 0.15 --step-forms $S_F32"
           "c4_rank_one:300:python3 bench.py --rccl-world1 $C4R --step-mode one"
           "c4_rank_perround:300:python3 bench.py --rccl-world1 $C4R --per-round-launches") ;;
  final)
    steps=("pytest_gpu:1100:$T -m gpu tests" "smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'"
           "bench_default:500:python3 bench.py" "prof_c3:900:scripts/profile_c3.sh $TAG $COMMIT") ;;
  step_alone)  # the one launch's cost while it runs alone: fully static steps, one round
    steps=("xi_alone4:300:$XI --config c4 --blocks '' --step-forms product,bf16_step_static_u8c4"
           "xi_alone4_forced:300:$XI --config c4 --blocks '' --forms bf16_bands4_u8c4,bf16_bands4_u8c2"
           "xi_alone1:300:$XI --config c4 --rounds 1 --blocks '' --step-forms product,bf16_step_static_u8c4") ;;
  e2e_c2)  # C2 end to end over chunk sizes x slots, two alternating passes
    steps=("e2e_c2_variants:900:for pass in 1 2; do for c in 32:3 64:3 64:4 16:4; do FEDAVG_STREAM_CHUNK_MB=\${c%:*} FEDAVG_STREAM_SLOTS=\${c#*:} python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 --no-cpu --check-cols 100000; done; done") ;;
  none) steps=() ;;
  *) echo "unknown recipe '$recipe'" >&2; exit 2 ;;
esac
exec scripts/gpu_steps.sh "${steps[@]}" "$@"
