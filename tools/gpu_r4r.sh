#!/bin/bash
# Round 4: the egress ordering check's connection table sized by the deliveries
# (GF_HZ_SIZED) and the LRU histogram grid at one block per CU (GF_LRU_BPC=1).
set -e
R=$(pwd)
O=$R/gpurun_out/r4r
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "egress or runtime_matrix or lru or config5" > "$O/tests.txt" 2>&1
echo "tests ok"
B=$R/tools/_bin
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_a.json" 2> "$O/eg_a.err"; echo ega
GPUFLOW_DIAG_LIB=$B/libgpuflow_hznosz.so timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_v.json" 2> "$O/eg_v.err"; echo egv
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_b.json" 2> "$O/eg_b.err"; echo egb
timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_a.json" 2> "$O/c5_a.err"; echo c5a
GPUFLOW_DIAG_LIB=$B/libgpuflow_lrubpc1.so timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_v.json" 2> "$O/c5_v.err"; echo c5v
timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2l_a.json" 2> "$O/c2l_a.err"; echo c2la
GPUFLOW_DIAG_LIB=$B/libgpuflow_lrubpc1.so timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2l_v.json" 2> "$O/c2l_v.err"; echo c2lv
echo "r4r done"
