set -e
O=gpurun_out/s5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "lru or gc or config5 or evict or fuzz" > $O/par.log 2>&1
echo parity-ok
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ks5 -o run -- python $R/bench.py --no-cpu --config 5 > $R/$O/b5.json 2> $R/$O/b5.err
echo prof-ok
