#!/bin/bash
# Reproduce the committed C3 profiles on an MI355X (run from the repo root, e.g. via gpurun):
#   scripts/gpu_steps.sh "prof:600:scripts/profile_c3.sh"
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (never combined with trace domains), then the traffic summary.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o c3 --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_c3_fetch" -o c3 -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_c3_write" -o c3 -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
cd "$ROOT"
python3 scripts/pmc_traffic.py --fetch "$OUT/pmc_c3_fetch" --write "$OUT/pmc_c3_write" \
    --kernel "k_fold_f32_gs<8, 4, true" --bytes 41000000000 --dispatches-per-call 3 --out profiles/pmc_c3.json
