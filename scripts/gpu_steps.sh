#!/bin/bash
# Run named GPU steps in order, each under its own time limit, logs in gpurun_out/.
# Usage: scripts/gpu_steps.sh "name:seconds:command" ...
# A step that exits 0 or 1 (test failures / Python errors) lets the next run;
# anything else (timeout 124/137, abort 134, segfault 139, ...) stops the call.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
    echo "== $name (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc in $(( $(date +%s) - start ))s"
    tail -n 5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping: $name ended with rc=$rc"
        exit $rc
    fi
done
