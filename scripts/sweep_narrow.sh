#!/bin/bash
# fp32 kernel-variant sweeps on narrow models (small P), where one lane per
# quad cannot fill 256 CUs: the LDS-staged fold (k_fold_f32_lds, variants
# lds_*) against the row-streaming fold.  Shapes: SURVEY.md App. D model sizes
# (speech CNN 67,267; MNIST CNN 582,026; Shakespeare LSTM 818,402; FEMNIST CNN
# 6,603,710) x client counts, plus BASELINE config 2.
#   bash scripts/sweep_narrow.sh   (on the GPU box, from the repo root)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep_table.log
: > "$out"
SHAPES=${SHAPES:-"1024:67267 256:67267 1024:582026 100:582026 1024:818402 100:1000000 1024:1000000 1024:2500000 1024:6603710"}
for shape in $SHAPES; do
    shape=${shape/:/ }
    set -- $shape
    echo "== clients $1 params $2" | tee -a "$out"
    timeout -k 10 150 python -u bench.py --config c2 --clients "$1" --params "$2" --sweep --steps 20 --warmup 2 \
        --no-cpu-baseline >> "$out" 2>&1 || exit $?
done
[ "${WITH_BASELINE_CONFIGS:-0}" = 1 ] || exit 0
for cfg in c3 c5; do  # the headline and the stall-aware config, same variant table
    echo "== config $cfg" | tee -a "$out"
    timeout -k 10 200 python -u bench.py --config $cfg --sweep --steps 8 --warmup 1 --no-cpu-baseline \
        >> "$out" 2>&1 || exit $?
done
