set -e
O=gpurun_out/s7; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_runtime_matrix.py -m gpu -x -v --timeout 300 --timeout-method thread -k "egress or trace or drop or matrix" > $O/par.log 2>&1
echo parity-ok
timeout -k 10 400 python -u bench.py --config egress > $O/beg.json 2> $O/beg.err
echo bench-ok
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kse -o run -- python $R/bench.py --no-cpu --config egress > $R/$O/kse.json 2>&1
echo prof-ok
