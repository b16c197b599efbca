#!/bin/bash
# Random-read rate against table footprint (tools/primbench.hip foot): where the L2
# and MALL steps sit, for the policy-layout question in DESIGN §8.
set -e
R=$(pwd); O=$R/gpurun_out/r4z; mkdir -p "$O"
timeout -k 10 180 "$R/tools/_bin/primbench" foot > "$O/primbench_foot.txt" 2>&1
echo "foot done"
