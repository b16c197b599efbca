#!/bin/bash
# Round 4: endpoint-class bucket lists per XCD (GF_NCLS), k_eg_front LDS sized by
# the snap (GF_EG_DYN), k_pipe_front at 8 waves (GF_FRONT_MINW) — the whole GPU
# suite, then A/B against the variants.
set -e
R=$(pwd)
O=$R/gpurun_out/r4l
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/tests.txt" 2>&1
echo "tests ok"
B=$R/tools/_bin
A="--no-cpu --no-extra --steps 8 --warmup 4 --long-steps 0"
timeout -k 10 200 python bench.py $A > "$O/c2_a.json" 2> "$O/c2_a.err"; echo c2a
GPUFLOW_DIAG_LIB=$B/libgpuflow_ncls1.so timeout -k 10 200 python bench.py $A > "$O/c2_v.json" 2> "$O/c2_v.err"; echo c2v
timeout -k 10 200 python bench.py $A > "$O/c2_b.json" 2> "$O/c2_b.err"; echo c2b
GPUFLOW_DIAG_LIB=$B/libgpuflow_ncls1.so timeout -k 10 200 python bench.py $A > "$O/c2_w.json" 2> "$O/c2_w.err"; echo c2w
for c in 4 5; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_a.json" 2> "$O/c${c}_a.err"; echo c${c}a
  GPUFLOW_DIAG_LIB=$B/libgpuflow_fminw8.so timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c${c}_v.json" 2> "$O/c${c}_v.err"; echo c${c}v
done
timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_a.json" 2> "$O/eg_a.err"; echo ega
GPUFLOW_DIAG_LIB=$B/libgpuflow_egstatic.so timeout -k 10 300 python bench.py --no-cpu --config egress > "$O/eg_v.json" 2> "$O/eg_v.err"; echo egv
echo "r4l done"
