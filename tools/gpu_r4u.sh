#!/bin/bash
# Round 4: the final tree — whole GPU suite and smoke, as the driver runs them.
set -e
R=$(pwd)
O=$R/gpurun_out/r4u
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/tests.txt" 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1; echo smoke
