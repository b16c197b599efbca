#!/bin/bash
# Round 4, first GPU call: the random-request ceiling matrix (tools/primbench.hip)
# with its request-size counters, then config 2 under the same counter passes
# (corrected HBM bytes and the L2 hit rate per kernel).
set -e
R=$(pwd)
O=$R/gpurun_out/r4a
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 "$R/tools/_bin/primbench" matrix > "$O/primbench.txt" 2>&1
echo "primbench done"
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum"
P2="TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"
P3="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$O/prim/p$i" -o run -- "$R/tools/_bin/primbench" matrix > "$O/prim_p$i.txt" 2>&1
  echo "primbench pmc pass $i done"
done
A="--no-cpu --no-extra --steps 4 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks2" -o run -- \
    python "$R/bench.py" $A > "$O/ks2.json" 2> "$O/ks2.err"
echo "config 2 kernel stats done"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$O/pmc2/p$i" -o run -- \
      python "$R/bench.py" $A > "$O/pmc2_p$i.json" 2> "$O/pmc2_p$i.err"
  echo "config 2 pmc pass $i done"
done
echo "r4a done"
