"""Ingest re-partition (cilium_amd.shard) on CPU: two gloo ranks
each receive an arbitrary half of every batch, move frames to the owner of
their flow group with one all-to-all, and classify what they hold through the
full pipeline; verdicts equal a single-process run over the same arrival
order, and the union of the ranks' CT partitions equals its CT."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cilium_amd import synth, shard, stream
from oracle.parity import owners_host  # noqa: F401  (the owner rule's host restatement)


def _ct_owner(k, world):
    if len(k) == 14:
        a = np.frombuffer(k[0:4], ">u4").astype(np.uint32)
        b = np.frombuffer(k[4:8], ">u4").astype(np.uint32)
        return int(stream.pair_rank(a, b, world)[0])
    return int(shard.pair_rank6(np.frombuffer(k[0:16], np.uint8)[None], np.frombuffer(k[16:32], np.uint8)[None],
                                world)[0])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.scenario import OracleDP
    sc = synth.pipeline_fuzz(seed=21, n_packets=6000, n_batches=2)
    ref, mine = OracleDP(sc), OracleDP(sc)
    for n in ("ct4", "ct6"):                       # a rank holds only its CT partition, pre-inserted entries too
        for k in list(mine.dump(n)):
            if _ct_owner(k, world) != rank:
                mine.m[n].delete(k)
    ok = True
    for bi, pk in enumerate(sc.batches):
        arrive = [np.nonzero(np.arange(pk.n) % world == s)[0] for s in range(world)]
        order_all = np.concatenate(arrive)                     # the node's arrival order: rank 0's, then rank 1's
        full = synth.Packets(*[None if x is None else x[order_all] for x in
                               (pk.frames, pk.lens, pk.src_identity, pk.ifindex, pk.lxc_id, pk.tc_index, pk.flow_hash)])
        ro, _, _ = ref.pipeline(full, sc.now + bi)
        # this rank's share of the arrivals, its owners, the exchange
        idx = arrive[rank]
        part = synth.Packets(*[None if x is None else x[idx] for x in
                               (pk.frames, pk.lens, pk.src_identity, pk.ifindex, pk.lxc_id, pk.tc_index, pk.flow_hash)])
        lo, nd6 = OracleDP.lb(mine, part)
        own = owners_host(lo, nd6, part, rank, world)
        order = np.argsort(own, kind="stable")
        counts = np.bincount(own, minlength=world)
        pos = sum(len(a) for a in arrive[:rank]) + np.arange(len(idx))   # position of each arrival in the node order
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
        got = shard.exchange(t(order), t(counts), [t(part.frames), t(part.lens.view(np.int32)), t(part.tc_index),
                                                   t(part.flow_hash.view(np.int32)), t(pos)])
        fr, ln, tci, fh, gpos = [x.numpy() for x in got]
        ln, fh = ln.view(np.uint32), fh.view(np.uint32)
        mo, _, _ = mine.pipeline(synth.Packets(fr, ln, None, None, None, tci, fh), sc.now + bi)
        ok &= bool(np.array_equal(mo, ro[gpos]))
    gathered = [None] * world
    dist.all_gather_object(gathered, {n: mine.dump(n) for n in ("ct4", "ct6")})
    ct_ok = True
    for n in ("ct4", "ct6"):
        union = {}
        for r, g in enumerate(gathered):
            ct_ok &= all(_ct_owner(k, world) == r for k in g[n])    # no entry on a rank that does not own it
            union.update(g[n])
        ct_ok &= union == ref.dump(n)
    q.put((rank, ok, ct_ok))
    dist.destroy_process_group()


def test_repartitioned_pipeline_matches_single_process():
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
    for rank, ok, ct_ok in res:
        assert ok, f"rank {rank}: verdicts differ from the single-process run"
        assert ct_ok, "union of per-rank CT partitions != single-process CT"
