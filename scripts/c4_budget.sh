#!/bin/bash
# Per-rank fold budget of the 8-GPU C4 step, measured on one GPU: the rank's
# 12.5M-param bf16 bucket (100M / 8) folded in R rounds of 12.5M/R-param slots
# with the RCCL all-gather of each round issued behind it (nccl at world 1 under
# torch.distributed.run: the exchange is a self-copy, so fold_ms is the
# per-rank fold time and gather_exposed_ms the non-overlapped tail), then the
# bf16 fold forms over those slot sizes (bench.py --sweep).
# Outputs: gpurun_out/c4_budget/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=${OUT:-gpurun_out/c4_budget}
mkdir -p "$OUT"
port=29611
for r in 1 2 4 8; do
  port=$((port + 1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --config c4 --params 12500000 --rounds $r --steps 30 --warmup 5 \
    --no-cpu-baseline > "$OUT/rounds$r.json" 2> "$OUT/rounds$r.err" || exit $?
  echo "rounds $r: $(python3 -c "import json; d=json.load(open('$OUT/rounds$r.json')); print('fold_ms', d['fold_ms'], 'exposed', d['gather_exposed_ms'], 'ms_per_step', d['ms_per_step'], 'gather_check', d['gather_check'])")"
done
for p in 12500000 6250000 3125000 1562500; do
  timeout -k 10 200 python bench.py --config c4 --params $p --sweep --steps 10 --warmup 2 --no-cpu-baseline \
    > "$OUT/sweep_$p.json" 2> "$OUT/sweep_$p.log" || exit $?
  echo "== bf16 256 x $p: $(grep -E '^variant' "$OUT/sweep_$p.log" | sort -t'>' -k2 -rn | head -4 | awk '{print $3, $5}' | tr '\n' ' ')"
done
