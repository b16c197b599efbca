import sys; sys.path.insert(0, '.')
import numpy as np, torch, struct
from cilium_amd import synth
from cilium_amd.datapath import Datapath, DeviceBatch, EG_OUT, to_numpy
from oracle.scenario import OracleDP
torch.cuda.set_device(0)
sc = synth.egress_fuzz(seed=6, n_packets=20000, n_batches=3, hazard=True)
dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
for bi, pk in enumerate(sc.batches):
    out, snap = dp.egress(DeviceBatch(pk, parse=False), sc.now + bi)
    torch.cuda.synchronize()
    ro, rs = ref.egress(pk, sc.now + bi)
    print("rec eq", np.array_equal(to_numpy(out, EG_OUT), ro))
    g, r = dp.dump_map("ct4"), ref.dump("ct4")
    print(bi, "ct eq", g == r)
    if g != r: break
def fmt(k): 
    d, s_, dp_, sp_, nh, fl = struct.unpack(">IIHHBB", k)
    return f"d={d:08x} s={s_:08x} dp={dp_} sp={sp_} nh={nh} fl={fl}"
only_g = set(g) - set(r); only_r = set(r) - set(g)
print("gpu only", len(only_g), "ref only", len(only_r))
for k in list(only_g)[:5]: print(" G", fmt(k), g[k].hex())
for k in list(only_r)[:5]: print(" R", fmt(k), r[k].hex())
diff = [k for k in set(g) & set(r) if g[k] != r[k]]
print("value diffs", len(diff))
for k in diff[:5]: print(" V", fmt(k), "\n   g", g[k].hex(), "\n   r", r[k].hex())
