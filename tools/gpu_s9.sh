set -e
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1
echo parity-ok
timeout -k 10 300 python -u bench.py --no-cpu --no-extra > $O/b2.json 2> $O/b2.err
echo bench-ok
