#!/bin/bash
set -e
O=gpurun_out/${1:-c4ab}; mkdir -p $O; V=${2:-fence}
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-h2d --config 4 > $O/cur$k.json 2> $O/cur$k.err
  GPUFLOW_DIAG_LIB=tools/_bin/libgpuflow_$V.so timeout -k 10 300 python -u bench.py --no-cpu --no-h2d --config 4 > $O/$V$k.json 2> $O/$V$k.err
  echo round-$k-ok
done
