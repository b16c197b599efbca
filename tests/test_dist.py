"""N>1 path on CPU (gloo, world_size 2): sharding packets by unordered address
pair (the bench's RSS-style partition) reproduces the single-process verdicts
and CT state exactly, and the counter all-reduce sums to the global counts."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cilium_amd import synth, stream


def _scenario():
    return synth.config2(n_flows=6000, n_pairs=800, n_ep=8, n_ids=128, n_l3=40, n_l4=80, n_wc=4, n_cidr=8,
                         ct_max=100000)


def _rank_of(pk, world):
    f = pk.frames
    sa = f[:, 26:30].copy().view(">u4").ravel()
    da = f[:, 30:34].copy().view(">u4").ravel()
    r = stream.pair_rank(sa.astype(np.uint32), da.astype(np.uint32), world)
    short = (pk.lens < 34) | (f[:, 12] != 0x08) | (f[:, 13] != 0x00)
    return np.where(short, np.arange(pk.n) % world, r)


def _key_rank(k, world):
    a = np.frombuffer(k[0:4], ">u4").astype(np.uint32)
    b = np.frombuffer(k[4:8], ">u4").astype(np.uint32)
    return int(stream.pair_rank(a, b, world)[0])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.scenario import OracleDP
    sc = _scenario()
    ref = OracleDP(sc)
    mine = OracleDP(sc)
    for k in list(mine.dump("cilium_ct4_global")):   # a rank holds only its CT partition
        if _key_rank(k, world) != rank:
            mine.m["cilium_ct4_global"].delete(k)
    res_ok = True
    counts = np.zeros(4, np.int64)
    for pk in sc.batches:
        full = ref.ingress(pk, sc.now)
        sel = np.nonzero(_rank_of(pk, world) == rank)[0]
        part = mine.ingress(_sub(pk, sel), sc.now)
        res_ok &= np.array_equal(part, full[sel])
        counts += np.bincount(part["ct_ret"], minlength=4)[:4]
    t = torch.from_numpy(counts)
    dist.all_reduce(t)                            # the bench's only collective (RCCL on GPUs)
    ct_mine = mine.dump("cilium_ct4_global")
    gathered = [None] * world
    dist.all_gather_object(gathered, ct_mine)
    union, owned = {}, True
    for r, g in enumerate(gathered):               # CT is partitioned: every entry on its owner only
        owned &= all(_key_rank(k, world) == r for k in g)
        union.update(g)
    ct_ok = owned and union == ref.dump("cilium_ct4_global")
    full_counts = np.zeros(4, np.int64)
    ref2 = OracleDP(sc)
    for pk in sc.batches:
        full_counts += np.bincount(ref2.ingress(pk, sc.now)["ct_ret"], minlength=4)[:4]
    q.put((rank, bool(res_ok), bool(ct_ok), bool(np.array_equal(t.numpy(), full_counts))))
    dist.destroy_process_group()


def _sub(pk, idx):
    f = lambda x: None if x is None else x[idx]
    return synth.Packets(pk.frames[idx], pk.lens[idx], f(pk.src_identity), f(pk.ifindex), f(pk.lxc_id),
                         f(pk.tc_index), f(pk.flow_hash))


def test_sharded_ingress_matches_single_process():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok, ct_ok, cnt_ok in res:
        assert ok, f"rank {rank}: verdicts differ from the single-process run"
        assert ct_ok, "union of per-rank CT partitions != single-process CT"
        assert cnt_ok, "all-reduced counters != global counts"
