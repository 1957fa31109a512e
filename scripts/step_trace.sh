#!/bin/bash
# Kernel trace of one rank's one-launch step under a one-rank RCCL group (C4 and C3 ranks):
# shows each round's all-gather kernel starting while the fold launch still runs.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/step_trace_c4 -o c4 --output-format csv -- python3 $R/bench.py --rccl-world1 --config c4 --params 12500000 --rounds 4 --steps 10 --warmup 3 --no-cpu-baseline --step-mode one > $R/gpurun_out/step_trace_c4.json 2> $R/gpurun_out/step_trace_c4.err && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/step_trace_c3 -o c3 --output-format csv -- python3 $R/bench.py --rccl-world1 --config c3 --rounds 4 --steps 10 --warmup 3 --no-cpu-baseline --step-mode one > $R/gpurun_out/step_trace_c3.json 2> $R/gpurun_out/step_trace_c3.err
