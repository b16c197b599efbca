#!/bin/bash
# Round profile of the bench workloads (run from the repo root on the GPU box):
#   1. rocprofv3 --kernel-trace --stats, one process per BASELINE configuration
#      (config 2 = the headline line; 1, 3, 4, 5, egress = the "configs" entries)
#   2. --pmc passes, one counter group per run (MI355X guide: FETCH_SIZE and
#      WRITE_SIZE in separate passes): the k_ing_groups request mix of config 2,
#      FETCH/WRITE of the roofline kernels of configs 1, 3, 4, 5
#   tools/profile_round.sh <tag>      -> gpurun_out/prof_<tag>/
#   CONFIGS="1 3" NO_C2=1 tools/profile_round.sh <tag>   (a subset)
set -e
CONFIGS=${CONFIGS:-"1 3 4 5 egress"}
T=${1:-r1}
R=$(pwd)
O=$R/gpurun_out/prof_$T
mkdir -p "$O" "$O/pmc"
cd /tmp && export TMPDIR=/tmp
if [ -z "$NO_C2" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks2" -o run -- \
    python "$R/bench.py" --no-cpu --no-extra > "$O/ks2.json" 2> "$O/ks2.err"
echo "kernel stats config 2 done"
fi
for C in $CONFIGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks$C" -o run -- \
      python "$R/bench.py" --no-cpu --config $C > "$O/ks$C.json" 2> "$O/ks$C.err"
  echo "kernel stats config $C done"
done
i=0
[ -n "$NO_C2" ] || for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_ATOMIC_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d "$O/pmc/c2/p$i" -o run -- \
      python "$R/bench.py" --no-cpu --no-extra --steps 2 --warmup 3 > "$O/pmc/c2p$i.json" 2> "$O/pmc/c2p$i.err"
  echo "config 2 pmc pass $i done"
done
for C in $CONFIGS; do
  i=0
  for P in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$O/pmc/c$C/p$i" -o run -- \
        python "$R/bench.py" --no-cpu --config $C > "$O/pmc/c${C}p$i.json" 2> "$O/pmc/c${C}p$i.err"
    echo "config $C pmc pass $i done"
  done
done
cd "$R"
if [ -z "$NO_C2" ]; then
python tools/pmc_summary.py "$O/pmc/c2" --steps 2 --out "$O/pmc_summary.json" > /dev/null
python tools/kstats.py "$O/ks2/run_kernel_stats.csv" 12 > "$O/kstats.txt"
fi
echo "summaries done"
