#!/bin/bash
# Reproduce the committed C3 profiles on an MI355X (run from the repo root, e.g. via gpurun):
#   scripts/gpu_steps.sh "prof:900:scripts/profile_c3.sh <tag> <commit>"
# the bench line itself, then kernel trace + stats of the same command, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (never combined with trace
# domains), then the traffic summary profiles/pmc_c3.json that bench.py reports
# as roofline.traffic.  Outputs: gpurun_out/prof_<tag>/.
set -euo pipefail
TAG=${1:-r02}
COMMIT=${2:-unknown}
# DPC: band dispatches per fold call (C3 with 3-pass bands: 4)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
# the trace and counter passes with the tuner off: its first call runs every
# candidate form once (C3: the gs kernel over other band and grid sizes among
# them), which would mix into the per-kernel averages and the per-dispatch
# counter medians; C3's measured form is the policy's gs_bands_16k anyway
# (bench.json config.fold_form), so the profiled kernel is the one the line times
export FEDAVG_AUTOTUNE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o c3 --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o c3 -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o c3 -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/write.err"
cd "$ROOT"
python3 scripts/pmc_traffic.py --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" \
    --kernel "k_fold_f32_gs<8, 4, true" --bytes 41000000000 --dispatches-per-call "${DPC:-4}" \
    --provenance "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (C3), round $TAG, commit $COMMIT, $(date -u +%Y-%m-%dT%H:%MZ)" \
    --out "$OUT/pmc_c3.json"
echo done
