#!/bin/bash
# The flow-group sort against the key bits it sorts (tools/sortbench.hip).
set -e
R=$(pwd); O=$R/gpurun_out/r4s2; mkdir -p "$O"
timeout -k 10 240 "$R/tools/_bin/sortbench" > "$O/sortbench.txt" 2>&1
echo "sortbench done"
