#!/bin/bash
# Round-end check at HEAD (run from the repo root on the GPU box): the GPU parity
# suite, the default bench line, then the config-2 + egress profile pass
# (kernel stats and FETCH/WRITE counters) of tools/profile_round.sh.
#   tools/gpu_round_r1c.sh <tag>      -> gpurun_out/<tag>/, gpurun_out/prof_<tag>/
set -e
T=${1:-r1c}
R=$(pwd)
O=$R/gpurun_out/$T
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
tail -3 "$O/gpu_tests.log"
timeout -k 10 500 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "bench done"
CONFIGS="egress" bash tools/profile_round.sh "$T"
