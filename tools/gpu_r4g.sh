#!/bin/bash
# Round 4: config-5 kernel timeline (host gaps), then the driver's default bench
# command end to end, timed.
set -e
R=$(pwd)
O=$R/gpurun_out/r4g
mkdir -p "$O"
CONFIGS=5 bash tools/gpu_trace.sh r4g
echo trace ok
S=$(date +%s)
timeout -k 10 800 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/full.json" 2> "$O/full.err"
echo "full bench $(( $(date +%s) - S )) s" | tee "$O/full.time"
