#!/bin/bash
# Wave priority in the grid-stride folds: the exchange interference proxy
# again, and the default bench line (no regression alone).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
exec scripts/gpu_steps.sh \
  "xi_c3:400:python3 tools/exchange_interference.py --config c3 --forms gs_bands_16k,dyn_8k,gs_bal_8k --blocks 16,32,64" \
  "xi_c4:300:python3 tools/exchange_interference.py --config c4 --blocks 16,32,64" \
  "bench_default:300:python3 bench.py --no-cpu-baseline"
