#!/bin/bash
# k_xdp_lds grid sweep on config 1 (GPU box): GF_XDP_GRID per run (0 = default).
set -e
O=gpurun_out/xdpgrid; mkdir -p $O
for rep in 1 2; do
  for g in 0 128 256 384 768 977 2048; do
    if [ $g = 0 ]; then e=""; else e="GF_XDP_GRID=$g"; fi
    env $e timeout -k 10 120 python bench.py --no-cpu --config 1 --steps 200 > $O/g${g}_$rep.json 2> $O/g${g}_$rep.err
  done
done
echo sweep-ok
