#!/bin/bash
# Round 4: egress — deferred-entry sets sized by the logged count, empty-family /
# no-IPv6 blocks skipped (GF_EG_LEAN) — egress GPU tests, egress A/B/A.
set -e
R=$(pwd)
O=$R/gpurun_out/r4o
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "egress or runtime_matrix or trace or drop" > "$O/tests.txt" 2>&1
echo "tests ok"
V=$R/tools/_bin/libgpuflow_eglegacy.so
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_a.json" 2> "$O/eg_a.err"; echo ega
GPUFLOW_DIAG_LIB=$V timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_v.json" 2> "$O/eg_v.err"; echo egv
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_b.json" 2> "$O/eg_b.err"; echo egb
echo "r4o done"
