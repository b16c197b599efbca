#!/bin/bash
# Host phase times per classify call (GF_HOST_PROF) of the config-5 and egress legs.
set -e
O=gpurun_out/${1:-hostprof}; mkdir -p $O
for C in ${CONFIGS:-5 egress}; do
  GF_HOST_PROF=1 timeout -k 10 300 python -u bench.py --no-cpu --config $C > $O/c$C.json 2> $O/c$C.err
  echo $C-ok
done
