#!/bin/bash
# A/B of the CT6 eviction histogram (full 64-B slots vs their second half,
# GF_LRU_V6HOT=1) on configuration 5, each with the LRU GPU tests; then the
# round's per-kernel profiles of configurations 2, 5 and egress at HEAD.
set -e
R=$(pwd); O=$R/gpurun_out/r3e; mkdir -p $O
GF_LRU_V6HOT=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_maps.py tests/test_gpu_scale.py -k "lru or config5" > $O/tests_v6hot.txt 2>&1
echo tests-ok
for M in full hot; do
  E=""; [ $M = hot ] && E=1
  (cd /tmp && export TMPDIR=/tmp && GF_LRU_V6HOT=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/ks5_$M -o run -- python $R/bench.py --config 5 > $O/c5_$M.json 2> $O/c5_$M.err)
  echo $M-ok
done
CONFIGS="2 5 egress" bash tools/profile_r3.sh r3b
