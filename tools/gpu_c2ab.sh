#!/bin/bash
# Same-box A/B of config 2: the tree's library vs a variant (tools/_bin), interleaved.
set -e
O=gpurun_out/${1:-c2ab}; mkdir -p $O; V=${2:-head}
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --no-extra --no-cpu > $O/cur$k.json 2> $O/cur$k.err
  GPUFLOW_DIAG_LIB=tools/_bin/libgpuflow_$V.so timeout -k 10 200 python -u bench.py --no-extra --no-cpu > $O/$V$k.json 2> $O/$V$k.err
  echo round-$k-ok
done
for C in egress 5; do
  timeout -k 10 300 python -u bench.py --no-cpu --config $C > $O/c$C.json 2> $O/c$C.err
  echo $C-ok
done
