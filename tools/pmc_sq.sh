#!/bin/bash
# SQ instruction-mix / wait-state passes over the bench (one counter group per run).
#   tools/pmc_sq.sh [outdir]     (repo root, GPU box)
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc_sq}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python "$R/bench.py" --no-cpu --steps 1 --warmup 3 > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  echo "pass $i done"
done
