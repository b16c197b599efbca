#!/bin/bash
# config-5 kernel trace (the CT6 eviction sweep every step), then the 1.07B-packet
# config-2 parity run (64 steps, sweeps from step ~20).
set -e
R=$(pwd); O=$R/gpurun_out/r3c; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks5 -o run -- \
    python $R/bench.py --no-cpu --config 5 > $O/c5.json 2> $O/c5.err)
echo c5-ok
bash tools/parity_1b.sh r3c_1b
echo all-ok
