set -e
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1
echo parity-ok
timeout -k 10 300 python -u bench.py --no-cpu > $O/b.json 2> $O/b.err
echo bench-ok
