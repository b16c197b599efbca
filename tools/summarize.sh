#!/bin/bash
# Host side of `tools/gpu.sh TAG prof:CFG ...`: per configuration the rocprofv3
# kernel stats and the per-kernel PMC summary (request-size bytes, request kinds,
# L2 hit rate, each kernel's rocprof average) into profiles/ROUND_*.
#   tools/summarize.sh TAG ROUND
set -e
T=$1; N=${2:-$1}
O=gpurun_out/$T
for P in "$O"/prof_*; do
  C=${P##*/prof_}
  [ -f "$P/ks/run_kernel_stats.csv" ] || continue
  cp "$P/ks/run_kernel_stats.csv" "profiles/${N}_kernel_stats_c$C.csv"
  cp "$P/ks.json" "profiles/${N}_bench_c$C.json"
  python tools/pmc_kernels.py "$P/pmc" --bench-json "$P/pmc/p1.json" --kernel-stats "$P/ks/run_kernel_stats.csv" \
      --out "profiles/${N}_pmc_kernels_c$C.json" > /dev/null
  echo "config $C summarized"
done
