#!/bin/bash
# Round 4: frame-staging loads issued together (GF_FRONT_UNROLL) in k_pipe_front /
# k_eg_front — pipeline / egress GPU tests, configs 4, 5 and egress against the
# one-load-at-a-time build; policy maps L2-resident ablation (GF_DIAG=32, diag).
set -e
R=$(pwd)
O=$R/gpurun_out/r4j
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "pipeline or egress or fuzz or config4 or trace or drop" > "$O/tests.txt" 2>&1
echo "tests ok"
B=$R/tools/_bin
for c in 4 5 egress; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_a.json" 2> "$O/c${c}_a.err"; echo c${c}a
  GPUFLOW_DIAG_LIB=$B/libgpuflow_fnounroll.so timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_v.json" 2> "$O/c${c}_v.err"; echo c${c}v
done
A="--no-cpu --no-extra --steps 8 --warmup 4 --long-steps 0"
GPUFLOW_DIAG_LIB=$B/libgpuflow_d32.so timeout -k 10 200 python bench.py $A > "$O/d32.json" 2> "$O/d32.err"; echo d32
timeout -k 10 200 python bench.py $A > "$O/base.json" 2> "$O/base.err"; echo base
echo "r4j done"
