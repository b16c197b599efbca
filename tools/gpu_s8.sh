set -e
O=gpurun_out/s8; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_runtime_matrix.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/par.log 2>&1
echo parity-ok
timeout -k 10 400 python -u bench.py --config egress --no-cpu > $O/beg.json 2> $O/beg.err
timeout -k 10 300 python -u bench.py --no-cpu --no-extra > $O/b2.json 2> $O/b2.err
echo bench-ok
for v in r11a r11b r8i24; do
  GPUFLOW_DIAG_LIB=$(pwd)/tools/_bin/libgpuflow_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-extra > $O/v_$v.json 2> $O/v_$v.err
done
echo variants-ok
