#!/bin/bash
# Host side of the round profile: per-configuration PMC summaries and kernel
# stats from gpurun_out/prof_<tag> (tools/profile_round.sh) into profiles/<tag>_*.
set -e
T=${1:-r2}
P=gpurun_out/prof_$T
python tools/kstats.py $P/ks2/run_kernel_stats.csv 12 > profiles/${T}_kstats.txt
cp $P/ks2/run_kernel_stats.csv profiles/${T}_kernel_stats.csv
cp $P/pmc_summary.json profiles/${T}_pmc_summary.json
for C in 1 3 4 5 egress; do
  cp $P/ks$C/run_kernel_stats.csv profiles/${T}_kernel_stats_c$C.csv
  read K NS NP <<< $(python - "$P/pmc/c${C}p1.json" "$C" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {"1": "k_xdp", "3": "k_lb"}.get(sys.argv[2], "gpuflow")
pk = {"1": 1000000, "3": 16000000, "4": 16777216}.get(sys.argv[2], 4194304)
print(k, d["steps"] + d["warmup"], pk)
PY
)
  python tools/pmc_summary.py $P/pmc/c$C --kernels $K --nsteps $NS --packets $NP --out profiles/${T}_pmc_summary_c$C.json > /dev/null
done
echo done
