#!/bin/bash
# Round 4: policy maps L2-resident ablation (GF_DIAG=32: every endpoint looks up
# program 0's map, counters in its own) against the product build, config 2.
set -e
R=$(pwd)
O=$R/gpurun_out/r4k
mkdir -p "$O"
A="--no-cpu --no-extra --steps 8 --warmup 4 --long-steps 0"
timeout -k 10 200 python bench.py $A > "$O/base_a.json" 2> "$O/base_a.err"; echo base_a
GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_d32.so timeout -k 10 200 python bench.py $A > "$O/d32.json" 2> "$O/d32.err"; echo d32
timeout -k 10 200 python bench.py $A > "$O/base_b.json" 2> "$O/base_b.err"; echo base_b
timeout -k 10 300 python bench.py --no-cpu --config 4 > "$O/c4.json" 2> "$O/c4.err"; echo c4
echo "r4k done"
