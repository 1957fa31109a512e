#!/bin/bash
# The ingest pipe after the abandoned-round drain and the per-device pool, its
# GPU tests and the e2e lines; the tuner's first-call cost on C3, C2 and a
# few-tile shape.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "ingest_tests:300:$PYT -m gpu tests/test_gpu_ingest.py tests/test_gpu_multigpu.py tests/test_gpu_dropin.py" \
  "first_call:300:FEDAVG_AUTOTUNE_LOG=1 python3 tools/tuner_probe.py --clients 1024 --params 10000000 && FEDAVG_AUTOTUNE_LOG=1 python3 tools/tuner_probe.py --clients 100 --params 1000000 && FEDAVG_AUTOTUNE_LOG=1 python3 tools/tuner_probe.py --clients 100 --params 300000 && FEDAVG_AUTOTUNE_LOG=1 python3 tools/tuner_probe.py --clients 256 --params 12500000 --bf16" \
  "e2e_lines:600:python3 bench_e2e.py --clients 10 --params 582026 --reps 20 && python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 && python3 bench_e2e.py --clients 100 --params 1000000 --reps 15 && python3 bench_e2e.py --clients 1024 --params 1000000 --reps 5"
