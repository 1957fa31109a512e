#!/bin/bash
# The measured form choice (tuner): its GPU tests, the whole GPU suite (every
# product fold now measures new shapes), the default bench line, the slot
# sweeps with the tuned auto fold, and the tail budget again.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
exec scripts/gpu_steps.sh \
  "tuner_tests:300:$PYT -m gpu tests/test_gpu_tuner.py" \
  "pytest_gpu:600:$PYT -m gpu tests" \
  "bench_default:300:python3 bench.py" \
  "slot_sweep:900:scripts/sweep_bf16_slots.sh" \
  "tail_budget:900:scripts/tail_budget.sh"
