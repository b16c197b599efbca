#!/bin/bash
# Random-read rate against table footprint (tools/primbench.hip foot) and per-XCD
# table slices against one shared table (xcd): the L2 / MALL steps behind the
# policy-layout question in DESIGN §8.   tools/gpu_r4z.sh [foot|xcd]
set -e
M=${1:-foot}
R=$(pwd); O=$R/gpurun_out/r4z; mkdir -p "$O"
timeout -k 10 180 "$R/tools/_bin/primbench" "$M" > "$O/primbench_$M.txt" 2>&1
echo "$M done"
