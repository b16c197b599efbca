#!/bin/bash
# Round 4: the driver's default bench command end to end on the profiled build
# (bounds from profiles/r4_pmc_kernels_c*.json of the same build id), timed.
set -e
R=$(pwd)
O=$R/gpurun_out/r4q
mkdir -p "$O"
S=$(date +%s)
timeout -k 10 800 python bench.py > "$O/full.json" 2> "$O/full.err"
echo "full bench $(( $(date +%s) - S )) s" | tee "$O/full.time"
