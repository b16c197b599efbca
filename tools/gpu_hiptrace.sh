#!/bin/bash
# HIP API + kernel timelines of bench legs (which host calls block, and where).
set -e
R=$(pwd); O=$R/gpurun_out/${1:-hiptrace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in ${CONFIGS:-5 egress}; do
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$O/ht$C" -o run -- \
      python "$R/bench.py" --no-cpu --config $C > "$O/ht$C.json" 2> "$O/ht$C.err"
  echo "hip trace $C done"
done
