#!/bin/bash
# k_lb stream-grid cap sweep on config 3 (GPU box): GPUFLOW_STREAM_GRID per run.
set -e
O=gpurun_out/lbgrid; mkdir -p $O
for g in 4096 8192 16384 32768; do
  GPUFLOW_STREAM_GRID=$g timeout -k 10 200 python bench.py --no-cpu --config 3 > $O/g$g.json 2> $O/g$g.err
done
echo sweep-ok
