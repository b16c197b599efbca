#!/bin/bash
# Per-kernel times of the LRU stand-in's eviction sweep at long horizons: config 2
# run long enough that the CT crosses max_entries (from step ~20) under
# rocprofv3 --kernel-trace --stats.  tools/gpu_lru_prof.sh <tag> [steps]
set -e
R=$(pwd); O=$R/gpurun_out/lru_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GF_LRU_STATS=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- \
    python $R/bench.py --no-cpu --no-extra --steps ${2:-36} --warmup 4 > $O/bench.json 2> $O/bench.err
cp $O/ks/*/run_kernel_stats.csv $O/kstats.csv 2>/dev/null || find $O/ks -name '*kernel_stats.csv' -exec cp {} $O/kstats.csv \;
echo lru-prof-ok
