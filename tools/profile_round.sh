#!/bin/bash
# Round profile of the bench workload (run from the repo root on the GPU box):
#   1. rocprofv3 --kernel-trace --stats over bench.py (per-kernel durations)
#   2. --pmc passes, one counter group per run (MI355X guide: FETCH_SIZE and
#      WRITE_SIZE in separate passes), for the k_ing_groups byte/request mix
#   3. primbench under FETCH_SIZE / WRITE_SIZE / EA requests (calibration)
#   tools/profile_round.sh <tag>      -> gpurun_out/prof_<tag>/
set -e
T=${1:-r1}
R=$(pwd)
O=$R/gpurun_out/prof_$T
mkdir -p "$O" "$O/pmc" "$O/cal"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks" -o run -- \
    python "$R/bench.py" --no-cpu --steps 4 > "$O/ks_bench.json" 2> "$O/ks_bench.err"
echo "kernel stats done"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_ATOMIC_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d "$O/pmc/p$i" -o run -- \
      python "$R/bench.py" --no-cpu --steps 2 --warmup 3 > "$O/pmc/p$i.json" 2> "$O/pmc/p$i.err"
  echo "pmc pass $i done"
done
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$O/cal/p$i" -o run -- "$R/tools/_bin/primbench" \
      > "$O/cal/p$i.txt" 2>&1
  echo "calibration pass $i done"
done
cd "$R"
python tools/pmc_summary.py "$O/pmc" --steps 2 --out "$O/pmc_summary.json" > /dev/null
python tools/kstats.py "$O/ks/run_kernel_stats.csv" 8 > "$O/kstats.txt"
echo "summaries done"
