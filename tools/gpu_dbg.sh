#!/bin/bash
set -e
O=gpurun_out/${1:-dbg}; mkdir -p $O
GF_SCHED=bins16 GF_SCHED_CHECK=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -v \
    --timeout 60 --timeout-method thread -s -k "fuzz_all_programs or elephant" > $O/t_bins16.txt 2>&1
echo bins16-check-ok
bash tools/gpu_ab.sh $1
