#!/bin/bash
# Default tail layouts per dtype (bench DEFAULT_TAIL) against equal rounds, and
# the slot sweeps with the tuned auto fold (bench pre-tunes before sweeping).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
exec scripts/gpu_steps.sh \
  "tail_budget:900:scripts/tail_budget.sh" \
  "slot_sweep:900:scripts/sweep_bf16_slots.sh"
