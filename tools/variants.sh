#!/bin/bash
# Build / time libgpuflow variants of compile-time tuning knobs with bench.py.
#   tools/variants.sh build "name:-DKNOB=v -DKNOB2=w" ...     (here)
#   tools/variants.sh run name ...                              (GPU box)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mode=$1; shift
if [ "$mode" = build ]; then
  mkdir -p "$R/tools/_bin"
  SHA=$(cd "$R" && python -c "import __graft_entry__ as g; print(g.source_sha())")
  for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DGF_SRC_SHA="\"$SHA+$name\"" $flags -I "$R/include" \
      "$R/cilium_amd/csrc/gf_maps.cpp" "$R/cilium_amd/csrc/gf_kernels.hip" -o "$R/tools/_bin/libgpuflow_$name.so" &
  done
  wait
  exit 0
fi
O=$R/gpurun_out/variants
mkdir -p "$O"
for name in "$@"; do
  GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$name.so timeout -k 10 200 python "$R/bench.py" \
      ${BENCH_ARGS:---no-cpu --no-extra --steps 8} > "$O/$name.json" 2> "$O/$name.err"
  echo "variant $name done"
done
