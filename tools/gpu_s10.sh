set -e
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread -k "xdp or config1 or fuzz or stream" > $O/par.log 2>&1
echo parity-ok
timeout -k 10 200 python -u bench.py --config 1 > $O/b1.json 2> $O/b1.err
GF_XDP_NOLDS=1 timeout -k 10 200 python -u bench.py --config 1 --no-cpu > $O/b1n.json 2> $O/b1n.err
echo bench-ok
