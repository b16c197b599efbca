#!/bin/bash
# Round 4: single-packet buckets in packet-index order in the egress passes
# (GF_SINGLE_ORDER) — whole GPU suite, egress A/B/A.
set -e
R=$(pwd)
O=$R/gpurun_out/r4v
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/tests.txt" 2>&1
echo "tests ok"
V=$R/tools/_bin/libgpuflow_single0.so
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_a.json" 2> "$O/eg_a.err"; echo ega
GPUFLOW_DIAG_LIB=$V timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_v.json" 2> "$O/eg_v.err"; echo egv
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_b.json" 2> "$O/eg_b.err"; echo egb
echo "r4v done"
