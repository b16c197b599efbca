#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace) of the egress and config-5 bench
# legs, for the host-gap analysis (tools/ktrace_gaps.py).
set -e
R=$(pwd); O=$R/gpurun_out/${1:-trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in ${CONFIGS:-egress 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt$C" -o run -- \
      python "$R/bench.py" --no-cpu --config $C > "$O/kt$C.json" 2> "$O/kt$C.err"
  echo "trace $C done"
done
