#!/bin/bash
# Round-end refresh (run from the repo root on the GPU box): the default bench line
# (config 2 + every configs entry), kernel stats of config 2 and of the egress leg,
# and the egress leg's FETCH_SIZE / WRITE_SIZE passes.   tools/gpu_round_r1b.sh <tag>
set -e
T=${1:-r1b}
R=$(pwd)
O=$R/gpurun_out/$T
mkdir -p "$O/pmc"
timeout -k 10 500 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "bench done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks2" -o run -- \
    python "$R/bench.py" --no-cpu --no-extra > "$O/ks2.json" 2> "$O/ks2.err"
echo "kernel stats config 2 done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kse" -o run -- \
    python "$R/bench.py" --no-cpu --config egress > "$O/kse.json" 2> "$O/kse.err"
echo "kernel stats egress done"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$O/pmc/ce/p$i" -o run -- \
      python "$R/bench.py" --no-cpu --config egress > "$O/pmc/cep$i.json" 2> "$O/pmc/cep$i.err"
  echo "egress pmc pass $i done"
done
