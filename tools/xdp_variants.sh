#!/bin/bash
# k_xdp (config 1) and k_pipe_front (config 4) under the XDP lookup variants
# built by tools/variants.sh build (GPU box).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/xdpv
mkdir -p "$O"
for rep in 1 2; do
  for name in "$@"; do
    GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$name.so timeout -k 10 120 python "$R/bench.py" --no-cpu --config 1 --steps 200 \
        > "$O/${name}_c1_$rep.json" 2> "$O/${name}_c1_$rep.err"
  done
done
for name in "$@"; do
  GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$name.so timeout -k 10 200 python "$R/bench.py" --no-cpu --config 4 \
      > "$O/${name}_c4.json" 2> "$O/${name}_c4.err"
  echo "variant $name done"
done
