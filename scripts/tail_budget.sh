#!/bin/bash
# Short-last-round layouts (bench.py --tail): per-rank fold cost of the 8-GPU
# C4 step (12.5M bf16 params x 256 clients) and of the 8-GPU C3 rank (10M fp32
# x 1024 clients, weak) in 4 rounds, the last round `tail` times the others,
# under nccl at world 1 (the gather is a self-copy: fold_ms is the real
# per-rank fold; the xGMI part of the exposed tail needs 8 GPUs).
# Outputs: gpurun_out/tail_budget/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/tail_budget}
mkdir -p "$OUT"
port=29711
run() {  # name, args...
  local name=$1; shift
  port=$((port + 1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit $?
  echo "$name: $(python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('widths', d['config']['round_widths'], 'fold_ms', d['fold_ms'], 'exposed', d['gather_exposed_ms'], 'ms_per_step', d['ms_per_step'], 'gather_check', d['gather_check'])")"
}
for pass in 1 2; do
  # equal rounds against the bench's default layout for the dtype (DEFAULT_TAIL) and the single-cut tails
  run "c4_equal_p$pass" --config c4 --params 12500000 --rounds 4 --tail 1 --steps 30 --warmup 5
  run "c4_default_p$pass" --config c4 --params 12500000 --rounds 4 --steps 30 --warmup 5
  run "c4_t0.125_p$pass" --config c4 --params 12500000 --rounds 4 --tail 0.125 --tail-steps 1 --steps 30 --warmup 5
  run "c3_equal_p$pass" --config c3 --rounds 4 --tail 1 --steps 10 --warmup 3
  run "c3_default_p$pass" --config c3 --rounds 4 --steps 10 --warmup 3
  run "c3_t0.125_p$pass" --config c3 --rounds 4 --tail 0.125 --tail-steps 1 --steps 10 --warmup 3
done
