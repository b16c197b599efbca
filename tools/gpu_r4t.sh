#!/bin/bash
# Round 4: DIR-24-8 through the pipeline front (GPU test), and the LRU histogram with
# 512-thread blocks, 3 a CU (GF_LRU_HB=512) on config 5 and the 64-step config 2.
set -e
R=$(pwd)
O=$R/gpurun_out/r4t
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
    -k "dir24" > "$O/tests.txt" 2>&1
echo "tests ok"
V=$R/tools/_bin/libgpuflow_lruhb512.so
timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_a.json" 2> "$O/c5_a.err"; echo c5a
GPUFLOW_DIAG_LIB=$V timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_v.json" 2> "$O/c5_v.err"; echo c5v
timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_b.json" 2> "$O/c5_b.err"; echo c5b
timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2l_a.json" 2> "$O/c2l_a.err"; echo c2la
GPUFLOW_DIAG_LIB=$V timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2l_v.json" 2> "$O/c2l_v.err"; echo c2lv
echo "r4t done"
