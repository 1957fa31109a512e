#!/bin/bash
# Opt-in split-client fold (fa_fedavg_f32_splitn, NOT bit-exact) against the
# exact auto fold on very narrow models.  Writes gpurun_out/splitn.log.
set -o pipefail
out=gpurun_out/splitn_table.log
: > "$out"
for shape in 1024:4096 1024:16384 1024:67267 256:67267 1024:582026; do
    n=${shape%%:*}; p=${shape##*:}
    for mode in exact splitn; do
        flag=""; [ $mode = splitn ] && flag="--splitn"
        line=$(timeout -k 10 120 python -u bench.py --config c2 --clients $n --params $p --steps 50 --warmup 5 \
               --no-cpu-baseline $flag 2>/dev/null) || exit $?
        echo "$n x $p $mode $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms_avg"], "ms", r["achieved"], "GB/s")')" >> "$out"
    done
done
cat "$out"
