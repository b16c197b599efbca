#!/bin/bash
# Round 4: k_pipe_front without its second header parse (GF_DIAG=64, diag) against
# the product build, configs 4 and 5.
set -e
R=$(pwd)
O=$R/gpurun_out/r4s
mkdir -p "$O"
V=$R/tools/_bin/libgpuflow_d64.so
for c in 4 5; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_a.json" 2> "$O/c${c}_a.err"; echo c${c}a
  GPUFLOW_DIAG_LIB=$V timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_v.json" 2> "$O/c${c}_v.err"; echo c${c}v
done
echo "r4s done"
