#!/bin/bash
# bf16 fold forms over the slot sizes that tail layouts produce for the 8-GPU
# C4 rank (12.5M params / rank, 256 clients; bench.py --sweep, config c4),
# and the fp32 forms over C3's tail slots (1024 clients).
# SHAPES_BF16 / SHAPES_F32 override.  Outputs: gpurun_out/bf16_slots/, gpurun_out/f32_slots/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export FEDAVG_AUTOTUNE_LOG=1  # the tuner's decisions (every candidate's time) go to the stderr logs
B=${B:-gpurun_out/bf16_slots}; F=${F:-gpurun_out/f32_slots}
mkdir -p "$B" "$F"
SHAPES_BF16=${SHAPES_BF16:-"256:961600 256:1136384 256:1250000 256:1500000 256:1785728 256:2000000 256:2272768 256:2500000 256:2750000 256:3125056 256:3571456 256:3846208 256:4545472"}
SHAPES_F32=${SHAPES_F32:-"1024:400000 1024:769280 1024:909120 1024:1818240 1024:2500032 1024:3076928 1024:3636352"}
for shape in $SHAPES_BF16; do
  n=${shape%%:*}; p=${shape##*:}
  timeout -k 10 240 python bench.py --config c4 --clients "$n" --params "$p" --sweep --steps 10 --warmup 2 \
    --no-cpu-baseline > "$B/${n}x${p}.json" 2> "$B/${n}x${p}.log" || exit $?
  echo "== bf16 ${n}x${p}: $(grep -E '^variant' "$B/${n}x${p}.log" | sort -t'>' -k2 -rn | head -3 | awk '{print $3, $5}' | tr '\n' ' ') auto: $(grep -E '^variant 0 ' "$B/${n}x${p}.log" | awk '{print $5}')"
done
for shape in $SHAPES_F32; do
  n=${shape%%:*}; p=${shape##*:}
  timeout -k 10 240 python bench.py --config c3 --clients "$n" --params "$p" --sweep --steps 8 --warmup 2 \
    --no-cpu-baseline > "$F/${n}x${p}.json" 2> "$F/${n}x${p}.log" || exit $?
  echo "== f32 ${n}x${p}: $(grep -E '^variant' "$F/${n}x${p}.log" | sort -t'>' -k2 -rn | head -3 | awk '{print $3, $5}' | tr '\n' ' ') auto: $(grep -E '^variant 0 ' "$F/${n}x${p}.log" | awk '{print $5}')"
done
