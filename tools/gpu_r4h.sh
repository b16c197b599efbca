#!/bin/bash
# Round 4: quad-cooperative slot reads in the LRU histogram (GF_LRU_COOP) and the
# cooperative CT6 probe at 3 waves (GF_CT_COOP6) — LRU GPU tests, config 5 and the
# 64-step config-2 run against the per-lane-load builds; policy-read ablations (diag);
# the egress CT4 probe by lane quads (GF_EG_COOP).
set -e
R=$(pwd)
O=$R/gpurun_out/r4h
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v \
    --timeout 240 --timeout-method thread -k "lru or config5 or egress or config2" > "$O/tests.txt" 2>&1
echo "tests ok"
B=$R/tools/_bin
timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_a.json" 2> "$O/c5_a.err"; echo c5a
GPUFLOW_DIAG_LIB=$B/libgpuflow_lrunocoop.so timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_v.json" 2> "$O/c5_v.err"; echo c5v
GPUFLOW_DIAG_LIB=$B/libgpuflow_coop6.so timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_c6.json" 2> "$O/c5_c6.err"; echo c5c6
timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_b.json" 2> "$O/c5_b.err"; echo c5b
timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2l_a.json" 2> "$O/c2l_a.err"; echo c2la
GPUFLOW_DIAG_LIB=$B/libgpuflow_lrunocoop.so timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2l_v.json" 2> "$O/c2l_v.err"; echo c2lv
A="--no-cpu --no-extra --steps 8 --warmup 4 --long-steps 0"
for v in d4 d16; do
  GPUFLOW_DIAG_LIB=$B/libgpuflow_$v.so timeout -k 10 200 python bench.py $A > "$O/$v.json" 2> "$O/$v.err"; echo $v
done
timeout -k 10 200 python bench.py $A > "$O/base.json" 2> "$O/base.err"; echo base
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_a.json" 2> "$O/eg_a.err"; echo ega
GPUFLOW_DIAG_LIB=$B/libgpuflow_egnocoop.so timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_v.json" 2> "$O/eg_v.err"; echo egv
echo "r4h done"
