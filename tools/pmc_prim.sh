#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / EA request calibration on primbench's known access
# counts (random 16-B loads, slot RMW, scatter) — one counter group per run.
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc_prim}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- "$R/tools/_bin/primbench" > "$OUT/p$i.txt" 2>&1
  echo "prim pass $i done"
done
