#!/bin/bash
# Round 4: cooperative CT home-line loads (GF_CT_COOP) — ingress parity on the GPU,
# then config 2 A/B/A against the per-lane load, config 5 with / without the CT6 form.
set -e
R=$(pwd)
O=$R/gpurun_out/r4c
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v --timeout 120 --timeout-method thread \
    -k "fuzz or config2 or elephant or pipeline or egress or lru or config5" > "$O/tests.txt" 2>&1
echo "tests ok"
A="--no-cpu --no-extra --steps 8 --warmup 4"
timeout -k 10 200 python bench.py $A > "$O/coop_a.json" 2> "$O/coop_a.err"; echo coop_a
GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_nocoop.so timeout -k 10 200 python bench.py $A > "$O/nocoop.json" 2> "$O/nocoop.err"; echo nocoop
timeout -k 10 200 python bench.py $A > "$O/coop_b.json" 2> "$O/coop_b.err"; echo coop_b
timeout -k 10 200 python bench.py --no-cpu --config 5 > "$O/c5.json" 2> "$O/c5.err"; echo c5
GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_coop6.so timeout -k 10 200 python bench.py --no-cpu --config 5 > "$O/c5_coop6.json" 2> "$O/c5_coop6.err"; echo c5coop6
echo "r4c done"
