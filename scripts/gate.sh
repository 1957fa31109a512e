#!/usr/bin/env bash
# Pre-commit gate: every Python file parses, the package imports, the CPU
# suite passes and build() compiles the gfx950 library.  Run before every
# commit (round 1 ended on a snapshot whose engine.py did not parse).
#   scripts/gate.sh          full gate
#   scripts/gate.sh --quick  parse + import only (seconds)
set -euo pipefail
cd "$(dirname "$0")/.."
python -m compileall -q fedlesscan_amd bench.py bench_e2e.py __graft_entry__.py tests oracle tools
python -c "import fedlesscan_amd, bench, bench_e2e"
if [[ "${1:-}" == "--quick" ]]; then
    echo "gate (quick): ok"
    exit 0
fi
python -c "import __graft_entry__ as g; g.build()"
python -m pytest tests -x -q -m "not gpu"
echo "gate: ok"
