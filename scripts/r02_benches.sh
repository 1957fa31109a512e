#!/bin/bash
# Every bench line DESIGN.md section 6 and the README quote, one gpurun call:
# the BASELINE configs and the narrow-model shapes (outputs in gpurun_out/benches/).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/benches
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  echo "== $n"
  timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>&1 || { echo "== $n failed"; tail -5 $O/$n.log; exit 1; }
  grep -o '"value": [0-9.]*' $O/$n.log | head -1
}
run c3 --gpus 1 --steps 20 --warmup 5
run c2 --config c2 --steps 200 --warmup 20 --no-cpu-baseline
run c4 --config c4 --steps 10 --warmup 2 --no-cpu-baseline
run c4b --config c4 --params 12500000 --steps 50 --warmup 5 --no-cpu-baseline
run c5 --config c5 --steps 10 --warmup 2 --no-cpu-baseline
for s in 1024:67267 256:67267 512:67267 100:67267 4096:67267 1024:16384 1024:40003 1024:98304 1024:131072 1024:200000 100:582026 10:582026 32:582026 64:582026 10:1000000 1024:786000 100:786000; do
  run small_${s/:/x} --config c3 --clients ${s%%:*} --params ${s##*:} --steps 200 --warmup 20 --no-cpu-baseline
done
echo done
