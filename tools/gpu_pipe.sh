set -e
O=gpurun_out/pipe1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "pipeline" > $O/par.log 2>&1
echo "pipeline parity ok"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/par_all.log 2>&1
echo "all gpu ok"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke ok"
