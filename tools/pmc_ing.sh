#!/bin/bash
# EA request mix of the ingress kernels (one counter group per rocprofv3 run).
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc_ing}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum" "TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python "$R/bench.py" --no-cpu --steps 2 --warmup 3 > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  echo "pass $i done"
done
