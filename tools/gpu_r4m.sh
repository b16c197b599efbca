#!/bin/bash
# Round 4: the settled build — whole GPU suite, smoke, then one bench line per
# configuration (no CPU leg).
set -e
R=$(pwd)
O=$R/gpurun_out/r4m
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/tests.txt" 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1; echo smoke
A="--no-cpu --no-extra --steps 8 --warmup 4 --long-steps 0"
timeout -k 10 200 python bench.py $A > "$O/c2.json" 2> "$O/c2.err"; echo c2
for c in 4 5 egress; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > "$O/c$c.json" 2> "$O/c$c.err"; echo c$c
done
echo "r4m done"
