#!/bin/bash
# Build and run tools/tuner_stress.cpp (the tuner's state machine against a
# simulated HIP runtime) under TSan, then ASan + UBSan (host only).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${TMPDIR:-/tmp}/fa_tuner_stress
mkdir -p "$OUT"
INC="-Itools/tunersim -Ifedlesscan_amd/csrc"
g++ -std=c++17 -O1 -g -fsanitize=thread $INC -o "$OUT/tsan" tools/tuner_stress.cpp -pthread
"$OUT/tsan"
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer $INC -o "$OUT/asan" tools/tuner_stress.cpp -pthread
"$OUT/asan"
