#!/bin/bash
# Round 4: page-translation sweep of the random line read (tools/primbench.hip tlb)
set -e
R=$(pwd)
O=$R/gpurun_out/r4b
mkdir -p "$O"
timeout -k 10 240 "$R/tools/_bin/primbench" tlb > "$O/tlb.txt" 2>&1
echo "tlb done"
