#!/bin/bash
# Ablation timing of k_ing_groups: builds libgpuflow variants with parts of the
# per-packet work compiled out (results are NOT valid verdicts) and times each
# with bench.py.  Build here:  tools/diag.sh build ;  run on the GPU box: tools/diag.sh run
#   GF_DIAG bits: 1 no output store, 2 no LDS stats, 4 no policy, 8 no CT create,
#                 16 no policy-map read (counters kept on a pseudo-random slot),
#                 32 every endpoint on program 0's policy map (one L2-resident table)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS=${VARIANTS:-"1 2 4 8 15"}
if [ "$1" = build ]; then
  mkdir -p "$R/tools/_bin"
  SHA=$(cd "$R" && python -c "import __graft_entry__ as g; print(g.source_sha())")
  for v in $VARIANTS; do
    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DGF_SRC_SHA="\"$SHA+d$v\"" -DGF_DIAG=$v -I "$R/include" \
      "$R/cilium_amd/csrc/gf_maps.cpp" "$R/cilium_amd/csrc/gf_kernels.hip" -o "$R/tools/_bin/libgpuflow_d$v.so" &
  done
  wait
  exit 0
fi
O=$R/gpurun_out/diag
mkdir -p "$O"
timeout -k 10 200 python "$R/bench.py" --no-cpu --steps 4 > "$O/base.json" 2>/dev/null
for v in $VARIANTS; do
  GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_d$v.so timeout -k 10 200 python "$R/bench.py" --no-cpu --steps 4 \
      > "$O/d$v.json" 2>/dev/null || echo "variant $v failed (verdict asserts may trip)"
  echo "variant $v done"
done
