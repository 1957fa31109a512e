#!/bin/bash
# Timeline of the end-to-end call (C2: 100 x 1M host NPZ blobs) with the native
# ingest pipe: kernel and memory-copy traces (no counters), analysed per round
# by scripts/e2e_timeline.py.  Outputs: gpurun_out/e2e_trace/
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/e2e_trace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/c2" -o run --output-format csv -- \
    python3 "$ROOT/bench_e2e.py" --clients 100 --params 1000000 --reps 15 --no-cpu > "$OUT/c2.json" 2> "$OUT/c2.err"
cd "$ROOT"
python3 scripts/e2e_timeline.py "$OUT/c2" > "$OUT/SUMMARY.md"
cat "$OUT/SUMMARY.md"
