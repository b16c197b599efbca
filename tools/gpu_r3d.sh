#!/bin/bash
# The GPU suite at HEAD, then an egress kernel trace (timeline gaps).
set -e
R=$(pwd); O=$R/gpurun_out/r3d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
echo tests-ok
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/egks -o run -- \
    python $R/bench.py --no-cpu --config egress > $O/eg.json 2> $O/eg.err)
echo trace-ok
GF_HOST_PROF=1 GF_SYNC_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --config egress > $O/eg_hp.json 2> $O/eg_hp.err
echo hostprof-ok
