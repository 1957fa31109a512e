#!/bin/bash
# The C3 fold split into R exchange rounds (the multi-GPU overlap structure),
# on one GPU: what splitting costs on the device side.  -> gpurun_out/rounds_table.log
set -o pipefail
out=gpurun_out/rounds_table.log
: > "$out"
for r in 1 2 4 8; do
    line=$(timeout -k 10 150 python -u bench.py --rounds $r --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null) || exit $?
    echo "rounds $r $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("fold per step", r["kernel_ms_avg"], "ms", r["achieved"], "GB/s")')" >> "$out"
done
cat "$out"
