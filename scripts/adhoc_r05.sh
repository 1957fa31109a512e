#!/bin/bash
# Round 5 A/B of the one-launch step kernel against another build of the repo
# (profiles/r05_step/kt_r04_vs_r05/): kernel traces of the C4-rank step run
# alone, alternating the two builds on one box.  OTHER names the other tree,
# copied into this one with its own built libraries (e.g. a round-4 checkout).
#   OTHER=ab_r04 /usr/local/graft/bin/gpurun --timeout 900 -- scripts/adhoc_r05.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OTHER=${OTHER:?set OTHER to the other tree}
OUT=$ROOT/gpurun_out/kt
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="--config c4 --blocks '' --steps 30 --step-forms product"
set -e
for run in other:$ROOT/$OTHER now:$ROOT other_b:$ROOT/$OTHER now_b:$ROOT; do
    name=${run%%:*}; tree=${run#*:}
    eval timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o kt --output-format csv -- \
        python3 "$tree/tools/exchange_interference.py" $A > "$OUT/$name.log" 2>&1
done
echo done
