#!/bin/bash
# k_xdp_lds staging budget sweep on config 1 (GPU box): GF_XDP_LDS_KB per run.
set -e
O=gpurun_out/xdpkb; mkdir -p $O
for rep in 1 2; do
  for kb in 16 32 48 80 96; do
    GF_XDP_LDS_KB=$kb timeout -k 10 120 python bench.py --no-cpu --config 1 --steps 200 > $O/kb${kb}_$rep.json 2> $O/kb${kb}_$rep.err
  done
  GF_XDP_NOLDS=1 timeout -k 10 120 python bench.py --no-cpu --config 1 --steps 200 > $O/nolds_$rep.json 2> $O/nolds_$rep.err
done
echo sweep-ok
