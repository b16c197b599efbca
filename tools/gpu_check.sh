#!/bin/bash
# GPU round trip used during development: parity tests, bench line, kernel stats.
#   tools/gpu_check.sh [tag]      (run from the repo root on the GPU box)
set -e
T=${1:-dev}
O=$(pwd)/gpurun_out/$T
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/par.log" 2>&1
echo "parity ok"
timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "bench ok"
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks" -o run -- python "$R/bench.py" --no-cpu --steps 4 > "$O/ks.json" 2>&1
echo "stats ok"
