#!/bin/bash
# The one runner for GPU calls (replaces the per-round tools/gpu_r*.sh one-offs,
# which are in git history).  Run from the repo root on the GPU box:
#
#   gpurun -- bash tools/gpu.sh TAG STEP [STEP ...]
#
# Every STEP runs under its own time limit and the first failing step ends the
# call (set -e): after a fault, an abort or a timeout nothing more touches the
# GPU.  Output goes to gpurun_out/TAG/.  A STEP is one word, its arguments
# separated by ':' (bench arguments by ',', e.g. bench:c2:--no-cpu,--steps,8):
#
#   tests[:EXPR]            pytest -m gpu [-k EXPR] ('+' for spaces)     -> tests.txt
#   smoke                   __graft_entry__.smoke()                      -> smoke.txt
#   bench:NAME[:ARGS]       python bench.py ARGS                         -> NAME.json, NAME.err
#   vbench:VAR:NAME[:ARGS]  bench.py on the variant library VAR (tools/variant.sh build VAR ...):
#                           a variant whose sources are not this tree's is rebuilt here first,
#                           from the flags it was built with (tools/_bin/libgpuflow_VAR.flags)
#   prof:CFG                rocprofv3 --kernel-trace --stats, then three --pmc passes (one counter
#                           group each) of bench configuration CFG       -> prof_CFG/
#   trace:NAME[:ARGS]       rocprofv3 --kernel-trace --stats of bench.py ARGS, the trace kept
#                           (tools/ktrace_gaps.py)                       -> trace_NAME/
#   primbench:MODE          tools/_bin/primbench MODE                    -> primbench_MODE.txt
#   pmc:CFG:C1,C2,..:NAME   one rocprofv3 --pmc pass (<= 8 SQ_, 4 TCC_ counters) of configuration CFG -> pmc_NAME/
#   env:K=V                 export K=V for the steps after it
#
# Host side afterwards: tools/summarize.sh TAG ROUND (profiles/ROUND_* from the prof steps' summaries).
set -e
T=$1; shift
R=$(pwd)
O=$R/gpurun_out/$T
mkdir -p "$O"
SHA=$(python -c "import __graft_entry__ as g; print(g.source_sha())")
args() { echo "$1" | tr ',' ' '; }

ensure_variant() {
  local v=$1 lib=$R/tools/_bin/libgpuflow_$1.so flags=$R/tools/_bin/libgpuflow_$1.flags
  if [ -f "$lib" ] && grep -qa "$SHA+$v" "$lib"; then return 0; fi
  [ -f "$flags" ] || { echo "variant $v: no library and no flags file"; return 1; }
  echo "variant $v: built from other sources, rebuilding here"
  timeout -k 10 400 hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DGF_SRC_SHA="\"$SHA+$v\"" \
      $(cat "$flags") -I "$R/include" "$R/cilium_amd/csrc/gf_maps.cpp" "$R/cilium_amd/csrc/gf_kernels.hip" -o "$lib"
}

prof() {
  local C=$1 P=$O/prof_$1 A
  if [ "$C" = 2 ]; then A="--no-cpu --no-extra --steps 4 --warmup 3 --long-steps 0"; else A="--no-cpu --config $C"; fi
  [ "$C" = 4 ] && A="$A --no-h2d"
  mkdir -p "$P/pmc"
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/ks" -o run -- \
       python "$R/bench.py" $A > "$P/ks.json" 2> "$P/ks.err")
  rm -f "$P/ks/run_kernel_trace.csv"                 # the stats stay; the trace would overflow gpurun_out
  echo "prof $C: kernel stats done"
  local i=0 G
  for G in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum" \
           "TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    (cd /tmp && export TMPDIR=/tmp &&
     timeout -s KILL 240 rocprofv3 --pmc $G --output-format csv -d "$P/pmc/p$i" -o run -- \
         python "$R/bench.py" $A > "$P/pmc/p$i.json" 2> "$P/pmc/p$i.err")
    echo "prof $C: pmc pass $i done"
  done
  # the per-dispatch counter CSVs of six configurations exceed what a call may bring
  # back (64 MiB): summarize here (tools/pmc_kernels.py, no GPU) and keep the summary
  python "$R/tools/pmc_kernels.py" "$P/pmc" --bench-json "$P/pmc/p1.json" --kernel-stats "$P/ks/run_kernel_stats.csv" \
      --out "$P/pmc_kernels.json" > "$P/pmc_kernels.txt"
  find "$P/pmc" -name '*.csv' -delete
  echo "prof $C: summarized"
}

for S in "$@"; do
  IFS=: read -r op a1 a2 a3 <<< "$S"
  case $op in
    tests)
      K=(); [ -n "$a1" ] && K=(-k "${a1//+/ }")        # '+' separates words: tests:lru+or+evict
      timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
          > "$O/tests.txt" 2>&1
      tail -1 "$O/tests.txt" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
      echo "smoke ok" ;;
    bench)
      timeout -k 10 900 python -u bench.py $(args "$a2") > "$O/$a1.json" 2> "$O/$a1.err"
      echo "bench $a1 ok" ;;
    vbench)
      ensure_variant "$a1"
      GPUFLOW_DIAG_LIB=$R/tools/_bin/libgpuflow_$a1.so timeout -k 10 900 python -u bench.py $(args "$a3") \
          > "$O/$a2.json" 2> "$O/$a2.err"
      echo "vbench $a1 $a2 ok" ;;
    prof)
      prof "$a1" ;;
    pmc)
      # one --pmc pass of bench configuration a1 with the counters a2 (comma-separated,
      # at most 8 SQ_ / 4 TCC_ ...: one pass, no splitting) -> pmc_NAME/ (a3 = NAME)
      P=$O/pmc_$a3; mkdir -p "$P"
      A="--no-cpu --config $a1"; [ "$a1" = 2 ] && A="--no-cpu --no-extra --steps 4 --warmup 3 --long-steps 0"
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -s KILL 240 rocprofv3 --pmc $(args "$a2") --output-format csv -d "$P/p1" -o run -- \
           python "$R/bench.py" $A > "$P/run.json" 2> "$P/run.err")
      python "$R/tools/pmc_kernels.py" "$P" --bench-json "$P/run.json" --out "$P/summary.json" > "$P/summary.txt" || true
      find "$P" -name '*counter_collection.csv' -size +20M -delete
      echo "pmc $a3 ok" ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$a1" -o run -- \
           python "$R/bench.py" $(args "$a2") > "$O/trace_$a1.json" 2> "$O/trace_$a1.err")
      echo "trace $a1 ok" ;;
    primbench)
      timeout -k 10 180 "$R/tools/_bin/primbench" "$a1" > "$O/primbench_$a1.txt" 2>&1
      echo "primbench $a1 ok" ;;
    env)
      export "$a1"; echo "env $a1" ;;
    *)
      echo "unknown step $S"; exit 2 ;;
  esac
done
echo "all steps done"
