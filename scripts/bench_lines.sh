#!/bin/bash
# Every bench line with the tuner on: C2, C3, C5, C4 whole model,
# C4 per-GPU bucket, and C3 / C4-bucket under a one-rank RCCL group with the
# default slot layouts.  Outputs: gpurun_out/benches/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export FEDAVG_AUTOTUNE_LOG=1  # the tuner's decisions (every candidate's time) go to the stderr logs
OUT=${OUT:-gpurun_out/benches}
mkdir -p "$OUT"
run() {  # name, seconds, args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit $?
  python3 - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]}: value {d['value']} GB/s, kernel {r['kernel_ms_avg']} ms, frac {r['frac']}, "
      f"of sweep {r['frac_of_read_ceiling']}, form {d['config'].get('fold_form')}, policy {d['config'].get('fold_policy')}, "
      f"step {d['ms_per_step']} ms, gather_check {d['gather_check']}")
PY
}
run c3 240
run c2 240 --config c2
run c5 240 --config c5
run c4_whole 240 --config c4
run c4_bucket 240 --config c4 --params 12500000
run c3_rccl_w1 240 --rccl-world1 --config c3 --no-cpu-baseline
run c4_bucket_rccl_w1 240 --rccl-world1 --config c4 --params 12500000 --no-cpu-baseline
