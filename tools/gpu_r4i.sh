#!/bin/bash
# Round 4: LDS frame rows padded to an odd word count in k_pipe_front / k_eg_front /
# k_eg_groups (GF_PIPE_PAD) — the whole GPU suite, then configs 4, 5 and egress
# against the unpadded build.
set -e
R=$(pwd)
O=$R/gpurun_out/r4i
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/tests.txt" 2>&1
echo "tests ok"
V=$R/tools/_bin/libgpuflow_nopad.so
for c in 4 5 egress; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_a.json" 2> "$O/c${c}_a.err"; echo c${c}a
  GPUFLOW_DIAG_LIB=$V timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_v.json" 2> "$O/c${c}_v.err"; echo c${c}v
done
echo "r4i done"
