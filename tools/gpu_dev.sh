#!/bin/bash
# development round trip: GPU parity (all), then the bench line (all configs)
#   tools/gpu_dev.sh tag
set -e
T=${1:-dev}
O=$(pwd)/gpurun_out/$T
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/par.log" 2>&1
echo "parity ok"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "bench ok"
