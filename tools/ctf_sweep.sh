#!/bin/bash
# CT slot factor variants (tools/variants.sh build): configs 2 and 5 (GPU box).
set -e
O=gpurun_out/ctf; mkdir -p $O
for name in f4 f2; do
  GPUFLOW_DIAG_LIB=tools/_bin/libgpuflow_$name.so timeout -k 10 300 python bench.py --no-cpu --no-extra > $O/${name}_c2.json 2> $O/${name}_c2.err
  GPUFLOW_DIAG_LIB=tools/_bin/libgpuflow_$name.so timeout -k 10 200 python bench.py --no-cpu --config 5 > $O/${name}_c5.json 2> $O/${name}_c5.err
  echo "$name done"
done
