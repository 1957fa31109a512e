#!/bin/bash
# Round-3 first GPU call: new multi-GPU / RCCL tests, the whole GPU suite,
# smoke, the default bench line, the RCCL bench at world 1 under
# torch.distributed.run, the self-launching 2-rank gloo rehearsal, and the
# bf16 counter passes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "new_tests:300:$PYT -m gpu tests/test_gpu_rccl.py tests/test_gpu_multigpu.py tests/test_handler_golden.py" \
  "gpu_suite:900:$PYT -m gpu tests" \
  "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_default:300:python3 bench.py" \
  "bench_rccl_w1:300:python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10" \
  "bench_gloo_w2:300:FEDAVG_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --config c3 --clients 64 --steps 2" \
  "bf16:900:scripts/profile_bf16.sh"
