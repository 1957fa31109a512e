#!/bin/bash
# Build and run tools/ingest_pipe_stress.cpp under TSan, then ASan + UBSan (host only).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${TMPDIR:-/tmp}/fa_ingest_stress
mkdir -p "$OUT"
SRC="tools/ingest_pipe_stress.cpp fedlesscan_amd/csrc/ingest_pipe.cpp"
INC="-Itools/hipsim -Iinclude -Ifedlesscan_amd/csrc"
g++ -std=c++17 -O1 -g -fsanitize=thread $INC -o "$OUT/tsan" $SRC -pthread
"$OUT/tsan"
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer $INC -o "$OUT/asan" $SRC -pthread
"$OUT/asan"
