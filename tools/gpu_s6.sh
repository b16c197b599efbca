set -e
O=gpurun_out/s6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_runtime_matrix.py -m gpu -x -v --timeout 300 --timeout-method thread -k "egress or trace or drop or matrix" > $O/par.log 2>&1
echo parity-ok
timeout -k 10 400 python -u bench.py --config egress > $O/beg.json 2> $O/beg.err
echo bench-ok
