#!/bin/bash
# Host side of tools/profile_r4.sh: kernel stats and per-kernel PMC summaries
# (corrected bytes, request kinds, L2 hit rate) into profiles/<tag>_*.
set -e
T=${1:-r4}
P=gpurun_out/prof_$T
for C in ${CONFIGS:-2 1 3 4 5 egress}; do
  [ -f $P/ks$C/run_kernel_stats.csv ] && cp $P/ks$C/run_kernel_stats.csv profiles/${T}_kernel_stats_c$C.csv
  [ -f $P/ks$C.json ] && cp $P/ks$C.json profiles/${T}_bench_c$C.json
  python tools/pmc_kernels.py $P/pmc/c$C --bench-json $P/pmc/c${C}p1.json --out profiles/${T}_pmc_kernels_c$C.json > /dev/null
done
python tools/kstats.py $P/ks2/run_kernel_stats.csv 7 > profiles/${T}_kstats.txt
echo done
