#!/bin/bash
# One bench configuration under libgpuflow variants built by tools/variants.sh build
# (GPU box):  tools/cfg_variants.sh CONFIG STEPS name ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cfg=$1; steps=$2; shift 2
O=$R/gpurun_out/cfgv
mkdir -p "$O"
for rep in 1 2; do
  for name in "$@"; do
    GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$name.so timeout -k 10 200 python "$R/bench.py" --no-cpu \
        --config "$cfg" --steps "$steps" > "$O/${name}_c${cfg}_$rep.json" 2> "$O/${name}_c${cfg}_$rep.err"
    echo "variant $name rep $rep done"
  done
done
