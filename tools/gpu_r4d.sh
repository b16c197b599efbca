#!/bin/bash
# Round 4: request sizes and rates of random reads/stores by cache policy
set -e
R=$(pwd)
O=$R/gpurun_out/r4d
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 "$R/tools/_bin/primbench" pol > "$O/pol.txt" 2>&1
echo "pol done"
i=0
for P in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum" \
         "TCC_EA0_WRREQ_64B_sum TCC_EA0_RD_UNCACHED_32B_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$O/pmc/p$i" -o run -- "$R/tools/_bin/primbench" pol > "$O/pmc_p$i.txt" 2>&1
  echo "pol pmc pass $i done"
done
