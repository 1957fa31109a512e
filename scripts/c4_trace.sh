#!/bin/bash
# Kernel trace of the 8-GPU C4 per-rank step on one GPU: the 12.5M-param bf16
# bucket in 4 rounds with the in-process one-rank RCCL group (bench.py
# --rccl-world1), so the timeline shows each round's fold, RCCL's kernels and
# the gaps between them.  Outputs: gpurun_out/c4_trace/
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/c4_trace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for r in 4 2; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/r$r" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config c4 --params 12500000 --rounds $r --rccl-world1 --steps 30 --warmup 5 \
      --no-cpu-baseline > "$OUT/r$r.json" 2> "$OUT/r$r.err"
done
cd "$ROOT"
ROUNDS=4 python3 scripts/trace_gaps.py "$OUT/r4" > "$OUT/SUMMARY.md"; ROUNDS=2 python3 scripts/trace_gaps.py "$OUT/r2" >> "$OUT/SUMMARY.md"
echo done
