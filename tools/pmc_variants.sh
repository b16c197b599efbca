#!/bin/bash
# EA read/write requests of k_ing_groups for libgpuflow variants (tools/variants.sh build ...):
#   tools/pmc_variants.sh base d1 d4 ...     (GPU box; "base" = the in-tree library)
set -e
R=$(pwd)
O=$R/gpurun_out/pmc_variants
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset GPUFLOW_DIAG_LIB; else export GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$v.so; fi
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d "$O/$v" -o run -- \
      python "$R/bench.py" --no-cpu --steps 2 --warmup 3 > "$O/$v.json" 2> "$O/$v.err"
  echo "variant $v done"
done
unset GPUFLOW_DIAG_LIB
cd "$R"
for v in "$@"; do mkdir -p "$O/$v/x" && mv "$O/$v/run_counter_collection.csv" "$O/$v/x/" && python tools/pmc_summary.py "$O/$v" --steps 2 --out "$O/$v.sum.json" > /dev/null; done
