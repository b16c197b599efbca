#!/bin/bash
# The north star's bit-exactness target on one MI355X: 64 config-2 steps of 16.8M
# packets (1.07B packets, 60 timed after 4 warm-up), every packet of every step and
# the CT at the end compared with the CPU oracle.
set -e
O=gpurun_out/${1:-parity1b}; mkdir -p $O
timeout -k 10 1150 python -u bench.py --no-extra --steps 60 --warmup 4 > $O/bench.json 2> $O/bench.err
echo parity-1b-ok
