#!/bin/bash
# Build libgpuflow variants here (hipcc cross-compiles gfx950); they travel to the
# GPU box with the tree (tools/_bin is git-ignored, not gpurun-ignored) and run
# through `tools/gpu.sh TAG vbench:NAME:OUT[:ARGS]`.  The flags are kept beside
# each library, so the runner can rebuild a variant the sources moved past.
#   tools/variant.sh NAME "-DKNOB=v -DKNOB2=w" [NAME2 "FLAGS2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/_bin"
SHA=$(cd "$R" && python -c "import __graft_entry__ as g; print(g.source_sha())")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  echo "$flags" > "$R/tools/_bin/libgpuflow_$name.flags"
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DGF_SRC_SHA="\"$SHA+$name\"" $flags -I "$R/include" \
    "$R/cilium_amd/csrc/gf_maps.cpp" "$R/cilium_amd/csrc/gf_kernels.hip" -o "$R/tools/_bin/libgpuflow_$name.so" &
done
wait
