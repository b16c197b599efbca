#!/bin/bash
# A/B of the schedule: parity tests of the ingress paths, then config 2 with the
# binned schedule (default), with records written in bucket order (GF_OUT_SORTED),
# and with the radix sort (GF_SCHED=radix).
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
GF_SCHED=bins timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "elephant or config2 or fuzz_all or pipelined or pipeline_fuzz or egress_fuzz" > $O/tests.txt 2>&1
echo tests-ok
GF_SCHED=bins GF_OUT_SORTED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "elephant or config2 or fuzz_all or pipelined" > $O/tests_os.txt 2>&1
echo tests-os-ok
GF_SCHED=bins timeout -k 10 300 python -u bench.py --no-extra --steps 8 --warmup 4 > $O/bin.json 2> $O/bin.err
echo bin-ok
GF_SCHED=bins GF_OUT_SORTED=1 timeout -k 10 300 python -u bench.py --no-extra --steps 8 --warmup 4 > $O/os.json 2> $O/os.err
echo os-ok
GF_SCHED=radix timeout -k 10 300 python -u bench.py --no-extra --no-cpu --steps 8 --warmup 4 > $O/radix.json 2> $O/radix.err
echo radix-ok
