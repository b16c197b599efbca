set -e
O=gpurun_out/s4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 250 --timeout-method thread -k "trace_notify or drop_notify or pipeline_fuzz or egress_fuzz or xdp" > $O/par.log 2>&1
echo parity-ok
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ks5 -o run -- python $R/bench.py --no-cpu --config 5 > $R/$O/b5.json 2> $R/$O/b5.err
echo prof-ok
