#!/bin/bash
# Round-3 GPU check: the parity suite, the default bench line (every config, parity
# over every pair), and the N-rank path rehearsed with two ranks sharing the GPU
# (gloo; RCCL itself needs one GPU per rank).   tools/gpu_r3.sh <tag> [steps...]
set -e
T=${1:-r3}; shift || true
STEPS=${@:-"tests bench ranks"}
O=gpurun_out/$T; mkdir -p $O
for S in $STEPS; do
  case $S in
    tests) timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
           echo tests-ok ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
           echo smoke-ok ;;
    bench) timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
           echo bench-ok ;;
    ranks) GPUFLOW_BENCH_BACKEND=gloo GPUFLOW_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 \
               --flows-per-step 1048576 --ct-max 33554432 --steps 4 --warmup 3 > $O/ranks2.json 2> $O/ranks2.err
           echo ranks-ok ;;
    variants) bash tools/variants.sh run $VARIANTS
           echo variants-ok ;;
  esac
done
