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
  if [ -f "$P/pmc_kernels.json" ]; then               # summarized on the box (tools/gpu.sh prof)
    cp "$P/pmc_kernels.json" "profiles/${N}_pmc_kernels_c$C.json"
  else
    python tools/pmc_kernels.py "$P/pmc" --bench-json "$P/pmc/p1.json" --kernel-stats "$P/ks/run_kernel_stats.csv" \
        --out "profiles/${N}_pmc_kernels_c$C.json" > /dev/null
  fi
  python - "profiles/${N}_pmc_kernels_c$C.json" "profiles/${N}_kernel_stats_c$C.csv" <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
j["kernel_stats_source"] = sys.argv[2]          # the copy in profiles/, not the box's path
json.dump(j, open(sys.argv[1], "w"), indent=1)
PY
  echo "config $C summarized"
done
