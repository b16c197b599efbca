set -e
mkdir -p gpurun_out/s2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_maps.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2/par.log 2>&1
echo parity-ok
for c in 1 5 4; do timeout -k 10 200 python -u bench.py --config $c --no-cpu > gpurun_out/s2/b$c.json 2> gpurun_out/s2/b$c.err; done
echo bench-ok
