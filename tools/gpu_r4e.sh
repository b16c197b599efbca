#!/bin/bash
# Round 4: nontemporal-load variants of the ingress kernel (config 2), then the
# driver's default bench command end to end (parity legs rewritten this round).
set -e
R=$(pwd)
O=$R/gpurun_out/r4e
mkdir -p "$O"
A="--no-cpu --no-extra --steps 8 --warmup 4"
timeout -k 10 200 python bench.py $A > "$O/base_a.json" 2> "$O/base_a.err"; echo base_a
for v in nt1 nt2 nt3; do
  GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$v.so timeout -k 10 200 python bench.py $A > "$O/$v.json" 2> "$O/$v.err"; echo $v
done
timeout -k 10 200 python bench.py $A > "$O/base_b.json" 2> "$O/base_b.err"; echo base_b
timeout -k 10 240 "$R/tools/_bin/primbench" pol > "$O/pol.txt" 2>&1; echo pol
/usr/bin/time -v timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/full.json" 2> "$O/full.err"; echo full
echo "r4e done"
