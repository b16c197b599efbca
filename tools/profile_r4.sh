#!/bin/bash
# Round-4 profile, per configuration (run from the repo root on the GPU box):
#   1. rocprofv3 --kernel-trace --stats of the bench configuration
#   2. three --pmc passes, one counter group per run:
#        request sizes: TCC_EA0_RDREQ + _32B + _128B, TCC_EA0_WRREQ
#        writes / L2:   TCC_EA0_WRREQ_64B, TCC_EA0_ATOMIC, TCC_HIT, TCC_MISS
#        issue:         SQ_INSTS_VALU + SALU + SQ_WAVES + GRBM_GUI_ACTIVE
#   tools/profile_r4.sh <tag>  -> gpurun_out/prof_<tag>/   (CONFIGS="2 5" for a subset)
#   host side: tools/profile_r4_summaries.sh <tag>
set -e
CONFIGS=${CONFIGS:-"2 1 3 4 5 egress"}
T=${1:-r4}
R=$(pwd)
O=$R/gpurun_out/prof_$T
mkdir -p "$O/pmc"
cd /tmp && export TMPDIR=/tmp
for C in $CONFIGS; do
  if [ "$C" = 2 ]; then A="--no-cpu --no-extra --steps 4 --warmup 3 --long-steps 0"; else A="--no-cpu --config $C"; fi
  [ "$C" = 4 ] && A="$A --no-h2d"                   # the H2D leg's extra steps would count twice
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks$C" -o run -- \
      python "$R/bench.py" $A > "$O/ks$C.json" 2> "$O/ks$C.err"
  rm -f "$O/ks$C/run_kernel_trace.csv"              # the stats are kept; the trace would overflow gpurun_out's 64 MiB
  echo "kernel stats config $C done"
  i=0
  for P in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum" \
           "TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$O/pmc/c$C/p$i" -o run -- \
        python "$R/bench.py" $A > "$O/pmc/c${C}p$i.json" 2> "$O/pmc/c${C}p$i.err"
    echo "config $C pmc pass $i done"
  done
done
echo "profile done"
