#!/bin/bash
# GF_PERM_VEC variants (tools/variants.sh build) on config 2 (GPU box).
set -e
O=gpurun_out/bw; mkdir -p $O
for rep in 1 2; do
  for name in bw0 bw1; do
    GPUFLOW_DIAG_LIB=tools/_bin/libgpuflow_$name.so timeout -k 10 300 python bench.py --no-cpu --no-extra > $O/${name}_$rep.json 2> $O/${name}_$rep.err
  done
done
echo sweep-ok
