#!/bin/bash
# LRU stand-in check: the eviction GPU tests, the sweep's kernel times at a long
# horizon, and config-2 parity over a run that evicts (every packet + the CT).
set -e
O=gpurun_out/lrucheck_${1:-a}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_maps.py tests/test_gpu_scale.py -k "lru or config5" > $O/tests.txt 2>&1
echo tests-ok
bash tools/gpu_lru_prof.sh ${1:-a} ${2:-36}
timeout -k 10 600 python -u bench.py --no-extra --steps ${2:-36} --warmup 4 > $O/parity.json 2> $O/parity.err
echo lru-check-ok
