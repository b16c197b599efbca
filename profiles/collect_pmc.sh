#!/bin/bash
# PMC passes for the bench's kernels (one counter group per rocprofv3 run, as the
# MI355X guide prescribes).  Run from the repo root on the GPU box:
#   profiles/collect_pmc.sh gpurun_out/pmc_r1
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc}
STEPS=${STEPS:-2}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_ATOMIC_sum"; do
  N=$(echo "$P" | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/$N" -o run -- \
      python "$R/bench.py" --no-cpu --steps "$STEPS" --warmup 3 > "$OUT/$N.json" 2> "$OUT/$N.err"
  echo "pass $N done"
done
