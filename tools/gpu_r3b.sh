#!/bin/bash
# Round-3 check after the LRU sweep rebuild: the eviction tests, then the full
# default bench (every configuration, parity legs, CPU baselines).
set -e
O=gpurun_out/r3b_${1:-a}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_maps.py tests/test_gpu_scale.py -k "lru or config5" > $O/tests.txt 2>&1
echo tests-ok
GF_LRU_STATS=1 timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-ok
