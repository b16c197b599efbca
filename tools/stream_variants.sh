#!/bin/bash
# Times the stream kernels (config 1 k_xdp, config 3 k_lb) for libgpuflow
# variants built by tools/variants.sh build (GPU box).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/variants
mkdir -p "$O"
for name in "$@"; do
  for cfg in 1 3; do
    GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$name.so timeout -k 10 200 python "$R/bench.py" --no-cpu --config $cfg \
        > "$O/${name}_c$cfg.json" 2> "$O/${name}_c$cfg.err"
  done
  echo "variant $name done"
done
