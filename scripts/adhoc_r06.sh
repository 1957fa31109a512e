#!/bin/bash
# Round 6 ad-hoc GPU steps (scripts/gpu_steps.sh): the product step against
# bench.py's loop, and the world-1 peer-copy decomposition.
C4R="--config c4 --params 12500000 --rounds 4 --steps 30 --warmup 5 --no-cpu-baseline"
C3R="--config c3 --rounds 4 --steps 20 --warmup 5 --no-cpu-baseline"
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
case "${1:-lines}" in
  tests)
    scripts/gpu_steps.sh "t_shared:400:$T tests/test_gpu_shared_fold.py" "t_sharding:500:$T tests/test_gpu_sharding.py" \
        "t_rccl:500:$T tests/test_gpu_rccl.py" ;;
  decomp)
    scripts/gpu_steps.sh "decomp_c4:300:python3 tools/peer_step_decomp.py --config c4" \
        "decomp_c3:300:python3 tools/peer_step_decomp.py --config c3 --steps 5" ;;
  lines)
    scripts/gpu_steps.sh \
     "c4r_prod_one_sync:300:python3 bench.py --rccl-world1 $C4R --step-mode one" \
     "c4r_prod_one_def:300:python3 bench.py --rccl-world1 $C4R --step-mode one --check deferred" \
     "c4r_loop_one:300:python3 bench.py --rccl-world1 $C4R --step-mode one --step-impl loop" \
     "c4r_prod_per:300:python3 bench.py --rccl-world1 $C4R --step-mode per-round" \
     "c4r_loop_per:300:python3 bench.py --rccl-world1 $C4R --step-mode per-round --step-impl loop" \
     "c4r_prod_peer:300:python3 bench.py --rccl-world1 $C4R --step-mode one --exchange peer_copy" \
     "c4r_prod_auto:300:python3 bench.py --rccl-world1 $C4R" \
     "c3r_prod_one_sync:300:python3 bench.py --rccl-world1 $C3R --step-mode one" \
     "c3r_prod_one_def:300:python3 bench.py --rccl-world1 $C3R --step-mode one --check deferred" \
     "c3r_loop_one:300:python3 bench.py --rccl-world1 $C3R --step-mode one --step-impl loop" \
     "c3r_prod_per:300:python3 bench.py --rccl-world1 $C3R --step-mode per-round" \
     "c3r_loop_per:300:python3 bench.py --rccl-world1 $C3R --step-mode per-round --step-impl loop" ;;
  probe)  # the warmed, pipelined step-form probe: what it chooses against both forms' lines
    scripts/gpu_steps.sh "t_sharding:500:$T tests/test_gpu_sharding.py" "t_rccl:500:$T tests/test_gpu_rccl.py" \
     "c4r_prod_auto:300:python3 bench.py --rccl-world1 $C4R" \
     "c3r_prod_auto:300:python3 bench.py --rccl-world1 $C3R" \
     "c4r_prod_one:300:python3 bench.py --rccl-world1 $C4R --step-mode one" \
     "c4r_prod_per:300:python3 bench.py --rccl-world1 $C4R --step-mode per-round" \
     "c3r_prod_one:300:python3 bench.py --rccl-world1 $C3R --step-mode one" \
     "c3r_prod_per:300:python3 bench.py --rccl-world1 $C3R --step-mode per-round" ;;
  c3one)  # the C3 rank's one launch: product vs loop vs the decomposition tool, one box
    scripts/gpu_steps.sh "c3r_prod_one:300:python3 bench.py --rccl-world1 $C3R --step-mode one" \
     "c3r_loop_one:300:python3 bench.py --rccl-world1 $C3R --step-mode one --step-impl loop" \
     "c3r_prod_per:300:python3 bench.py --rccl-world1 $C3R --step-mode per-round" \
     "decomp_c3:300:python3 tools/peer_step_decomp.py --config c3 --steps 5 --only fold_agent,product_rccl,product_sync" ;;
  hops)  # what the bench's per-fold events and the caller-stream hops add to the product step
    scripts/gpu_steps.sh "hops_c4:300:python3 tools/peer_step_decomp.py --config c4 --only fold_agent,product_rccl,product_per,product_rccl_traced,product_per_traced,product_rccl_dflt,product_per_dflt" \
     "hops_c3:300:python3 tools/peer_step_decomp.py --config c3 --steps 5 --only fold_agent,product_rccl,product_per,product_rccl_traced,product_per_traced,product_rccl_dflt,product_per_dflt" ;;
  capture)  # captured graphs replayed over fresh rows
    scripts/gpu_steps.sh "t_capture:300:$T tests/test_gpu_sharding.py -k 'captured_graph or captures_into'" ;;
  trace)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/tr_peer" \
        -o peer --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/peer_step_decomp.py" \
        --only fold_sys,peer_step,product_peer,product_rccl --reps 2 --steps 5 ;;
esac
