set -e
O=gpurun_out/s11; mkdir -p $O
for kb in 144 16 48; do
  GF_XDP_LDS_KB=$kb timeout -k 10 200 python -u bench.py --config 1 --no-cpu --steps 200 > $O/b1_$kb.json 2> $O/b1_$kb.err
done
GF_XDP_NOLDS=1 timeout -k 10 200 python -u bench.py --config 1 --no-cpu --steps 200 > $O/b1_n.json 2> $O/b1_n.err
echo bench-ok
