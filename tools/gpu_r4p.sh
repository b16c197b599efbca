#!/bin/bash
# Round 4: the settled build — whole GPU suite, smoke, config 5 with the count
# readbacks printed (GF_SYNC_DEBUG), egress.
set -e
R=$(pwd)
O=$R/gpurun_out/r4p
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/tests.txt" 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1; echo smoke
GF_SYNC_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5.json" 2> "$O/c5.err"; echo c5
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg.json" 2> "$O/eg.err"; echo eg
echo "r4p done"
