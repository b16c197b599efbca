#!/bin/bash
# Egress / config-5 checks: parity tests, the legs with sync debug, config 2, timelines.
set -e
O=gpurun_out/${1:-eg}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "${TESTS:-egress or runtime or trace or maps or pipeline or scale}" > $O/gpu_tests.txt 2>&1
echo tests-ok
for C in egress 5; do
GF_SYNC_DEBUG=1 timeout -k 10 300 python -u bench.py --config $C > $O/c$C.json 2> $O/c$C.err
echo $C-ok
done
timeout -k 10 300 python -u bench.py --no-extra --no-cpu > $O/c2.json 2> $O/c2.err
echo c2-ok
CONFIGS="egress 5" bash tools/gpu_trace.sh ${1:-eg}
