#!/bin/bash
# A/B: parity tests under GF_SCHED=bins16, config 2 with bins16 / radix, and the
# memo-size variants (tools/variants.sh).
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
GF_SCHED=bins16 GF_SCHED_CHECK=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "elephant or fuzz_all" > $O/tests_check.txt 2>&1
echo check-ok
GF_SCHED=bins16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "elephant or config2 or fuzz_all or pipelined or pipeline_fuzz or egress_fuzz" > $O/tests_bins16.txt 2>&1
echo tests-bins16-ok
GF_SCHED=bins16 timeout -k 10 300 python -u bench.py --no-extra --no-cpu --steps 8 --warmup 4 > $O/bins16.json 2> $O/bins16.err
echo bins16-ok
timeout -k 10 300 python -u bench.py --no-extra --no-cpu --steps 8 --warmup 4 > $O/radix.json 2> $O/radix.err
echo radix-ok
bash tools/variants.sh run memo3 memo4
cp gpurun_out/variants/memo*.json $O/
