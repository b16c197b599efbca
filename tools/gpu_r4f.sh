#!/bin/bash
# Round 4: partial LRU sweeps — GPU tests (LRU, config 5 real shape, ingress and
# egress parity), config 5 and the config-2 long horizon with partial vs whole-table
# sweeps, then the driver's default bench command end to end.
set -e
R=$(pwd)
O=$R/gpurun_out/r4f
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 240 \
    --timeout-method thread -k "lru or config5 or fuzz or config2 or egress or pipeline or dir24 or xdp" > "$O/tests.txt" 2>&1
echo "tests ok"
timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5.json" 2> "$O/c5.err"; echo c5
GF_LRU_FULL=1 timeout -k 10 300 python bench.py --no-cpu --config 5 > "$O/c5_full.json" 2> "$O/c5_full.err"; echo c5full
timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2long.json" 2> "$O/c2long.err"; echo c2long
GF_LRU_FULL=1 timeout -k 10 300 python bench.py --no-cpu --no-extra > "$O/c2long_full.json" 2> "$O/c2long_full.err"; echo c2longfull
for c in 1 4; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c$c.json" 2> "$O/c$c.err"; echo c$c
  GF_XDP_DIR24=1 timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_dir.json" 2> "$O/c${c}_dir.err"; echo c${c}dir
done
echo "r4f done"
