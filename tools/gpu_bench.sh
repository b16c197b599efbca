#!/bin/bash
# bench (all configs) + parity, development round trip:  tools/gpu_bench.sh tag
set -e
T=${1:-dev}
O=$(pwd)/gpurun_out/$T
mkdir -p "$O"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "bench ok"
