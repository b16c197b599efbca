#!/bin/bash
# Quick perf check of every leg without parity (and the GPU tests named in $TESTS).
set -e
O=gpurun_out/${1:-quick}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" > $O/gpu_tests.txt 2>&1
  echo tests-ok
fi
timeout -k 10 600 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
echo bench-ok
