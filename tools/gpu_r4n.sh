#!/bin/bash
# Round 4: egress log sizes per call (GF_EG_LOGSTATS) and the egress kernel timeline.
set -e
R=$(pwd)
O=$R/gpurun_out/r4n
mkdir -p "$O"
GF_EG_LOGSTATS=1 timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_logstats.json" 2> "$O/eg_logstats.err"; echo logstats
CONFIGS=egress bash tools/gpu_trace.sh r4n
echo "r4n done"
