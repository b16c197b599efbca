#!/bin/bash
# Round-4 final-tree check: the whole GPU suite, smoke, and the N-rank bench path
# rehearsed with two ranks sharing the one GPU (gloo collectives; RCCL needs a GPU
# per rank): config 2 and config 4's owned / exchange legs through the real kernels.
set -e
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo smoke-ok
GPUFLOW_BENCH_BACKEND=gloo GPUFLOW_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 \
    --flows-per-step 1048576 --ct-max 33554432 --steps 4 --warmup 3 > $O/ranks2.json 2> $O/ranks2.err
echo ranks-ok
