#!/bin/bash
# Round-end check at HEAD: smoke(), then the default bench (every configuration).
set -e
O=gpurun_out/final_${1:-a}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo smoke-ok
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-ok
