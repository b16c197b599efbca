#!/bin/bash
# Round-end GPU run part 1: the GPU parity suite and the default bench line
# (every configuration with its CPU baseline and parity leg).
set -e
O=gpurun_out/final; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo parity-ok
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo bench-ok
