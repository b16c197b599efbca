"""Per-endpoint CT maps — the ConntrackLocal endpoint option
(pkg/endpoint/bpf.go:268-276: `#define CT_MAP4 cilium_ct4_<id>` instead of
cilium_ct4_global; bpf/lxc_config.h:38-40 is the reference's own per-endpoint
template).  The reference's RuntimeValidatedConntrackTest runs its matrix with the
option disabled and enabled (test/runtime/connectivity.go:672-690).

CPU: the oracle's per-endpoint semantics (each program's CT_MAP4 / CT_MAP6, bpf_lxc.c
ct_lookup4/ct_create4 on &CT_MAP4).  GPU: libgpuflow's per-endpoint kernels
(k_ing_groups<FAM, 1, true>) against the oracle, records and every CT map bit-exact.
"""

import numpy as np
import pytest

from cilium_amd import synth
from cilium_amd.synth import Packets
from oracle.scenario import OracleDP


def _subset(pk, m):
    f = lambda x: None if x is None else x[m]
    return Packets(pk.frames[m], pk.lens[m], f(pk.src_identity), f(pk.ifindex), f(pk.lxc_id), f(pk.tc_index),
                   f(pk.flow_hash))


def test_conntrack_local_maps_are_independent():
    """With every endpoint on its own CT maps, one endpoint's packets classified alone
    give the same records and the same CT maps as inside the whole batch: nothing
    another endpoint does reaches its conntrack state (oracle, 3 batches, LRU on)."""
    sc = synth.fuzz(seed=21, n_packets=6000, n_batches=3)
    made = synth.conntrack_local(sc, max_entries=1500)
    assert len(made) == 2 * len(sc.lxc)
    ids = [e["lxc_id"] for e in sc.lxc]
    whole = OracleDP(sc)
    recs = [whole.ingress(pk, sc.now + bi) for bi, pk in enumerate(sc.batches)]
    for lid in ids[:4]:
        alone = OracleDP(sc)
        for bi, pk in enumerate(sc.batches):
            m = pk.lxc_id == lid
            got = alone.ingress(_subset(pk, m), sc.now + bi)
            assert np.array_equal(got, recs[bi][m]), f"endpoint {lid} batch {bi}"
        for fam in ("ct4", "ct6"):
            assert alone.dump(f"{fam}_{lid}") == whole.dump(f"{fam}_{lid}"), f"{fam}_{lid}"
    # the local maps did fill (and evict) on their own
    sizes = [len(whole.dump(f"ct4_{lid}")) for lid in ids]
    assert max(sizes) > 0 and max(sizes) <= 1500


def test_conntrack_local_mixed_keeps_global_for_the_rest():
    """Half of the endpoints local: the other half's entries stay in the shared map,
    the local ones' in theirs (oracle)."""
    sc = synth.fuzz(seed=22, n_packets=6000, n_batches=2)
    pre = len(sc.maps["ct4"].keys)
    synth.conntrack_local(sc, every=2)
    ref = OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        ref.ingress(pk, sc.now + bi)
    local = [e["lxc_id"] for j, e in enumerate(sc.lxc) if j % 2 == 0]
    assert all(sc.lxc[j]["ct4"] == "ct4" for j in range(1, len(sc.lxc), 2))
    grew = [len(ref.dump(f"ct4_{lid}")) > pre for lid in local]
    assert any(grew)


# ---------------------------------------------------------------- GPU parity
torch = pytest.importorskip("torch")


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,every,mx", [(1, 1, None), (2, 2, None), (3, 1, 700), (4, 3, 1200)])
def test_gpu_conntrack_local_ingress(seed, every, mx):
    """handle_policy with per-endpoint CT maps (all, every 2nd, every 3rd endpoint; small
    max_entries: each map's own LRU eviction): records and every CT map equal the
    oracle's, batch after batch."""
    _gpu()
    from cilium_amd.datapath import Datapath, DeviceBatch, ING_OUT, to_numpy
    sc = synth.fuzz(seed=seed, n_packets=20000, n_batches=3)
    made = synth.conntrack_local(sc, every=every, max_entries=mx)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        io = dp.ingress(DeviceBatch(pk), sc.now + bi)
        torch.cuda.synchronize()
        got, want = to_numpy(io, ING_OUT), ref.ingress(pk, sc.now + bi)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, f"batch {bi}: {len(bad)} records differ, first {bad[:1]}"
    for name in made + ["ct4", "ct6"]:
        assert dp.dump_map(name) == ref.dump(name), name
    for e in range(16):
        assert dp.dump_map(f"pol{e}") == ref.dump(f"pol{e}"), f"pol{e}"
    if mx:
        evicted = [n for n in made if n.startswith("ct4_") and len(ref.dump(n)) <= mx]
        assert evicted, "the small local maps should have been held at max_entries"


@pytest.mark.gpu
@pytest.mark.parametrize("seed,every", [(3, 1), (8, 2)])
def test_gpu_conntrack_local_pipeline(seed, every):
    """The full pipeline (XDP -> LB -> netdev -> handle_policy) with per-endpoint CT
    maps: records, rewritten frames and every CT map equal the oracle's."""
    _gpu()
    from cilium_amd.datapath import Datapath, DeviceBatch, PIPE_OUT, to_numpy
    sc = synth.pipeline_fuzz(seed=seed, n_packets=20000, n_batches=3)
    made = synth.conntrack_local(sc, every=every)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        out, nd6, snap = dp.pipeline(DeviceBatch(pk, parse=False), sc.now + bi)
        torch.cuda.synchronize()
        ro, rn6, rs = ref.pipeline(pk, sc.now + bi)
        got = to_numpy(out, PIPE_OUT)
        assert np.array_equal(got, ro), f"pipeline b{bi}"
        assert np.array_equal(nd6.cpu().numpy(), rn6), f"nd6 b{bi}"
        assert not (snap.cpu().numpy() != rs).any(), f"frames b{bi}"
    for name in made + ["ct4", "ct6"]:
        assert dp.dump_map(name) == ref.dump(name), name
    assert dp.dump_map("cilium_proxy4") == ref.dump("cilium_proxy4")


@pytest.mark.gpu
@pytest.mark.parametrize("n_ep,mx", [(40, 1500), (20, 600)])
def test_gpu_conntrack_local_many_maps(n_ep, mx):
    """More per-endpoint maps than one multi-map eviction chain takes (GF_LRU_MULTI = 32:
    40 maps run as chains of 32 and 8), each small enough to evict on every call:
    the config-2 stream in four calls, records and all 40 maps equal the oracle's."""
    _gpu()
    from cilium_amd.datapath import Datapath, DeviceBatch, ING_OUT, to_numpy
    sc = synth.config2(n_flows=120_000, n_pairs=12_000, n_ep=n_ep, n_ids=512, n_l3=200, n_l4=400, n_wc=8,
                       n_cidr=32, ct_max=400_000)
    made = synth.conntrack_local(sc, max_entries=mx)
    assert len(made) == n_ep
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    q = (pk.n + 3) // 4
    for k in range(4):
        part = pk.slice(k * q, min(pk.n, (k + 1) * q))
        io = dp.ingress(DeviceBatch(part), sc.now + k)
        torch.cuda.synchronize()
        got, want = to_numpy(io, ING_OUT), ref.ingress(part, sc.now + k)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, f"call {k}: {len(bad)} records differ, first {bad[:1]}"
    for name in made:
        assert dp.dump_map(name) == ref.dump(name), name
    # every map evicted after every call (a map holding more than one call's inserts
    # also ends at or below max_entries: include/gpuflow.h's bound)
    assert all(len(ref.lru_log[name]) == 4 for name in made), {n: len(ref.lru_log[n]) for n in made}


@pytest.mark.gpu
@pytest.mark.parametrize("every,mx", [(1, 500), (2, 800)])
def test_gpu_conntrack_local_queued_calls(every, mx):
    """Eight calls queued back to back, no host sync between them, on 40 small
    per-endpoint maps (all or every 2nd endpoint; the rest on the global map): the host's
    count bound of each map refreshes only from the counts the multi-map eviction pass
    stamps (`seq << 32 | count`), which may be a call or more behind the host.  Every
    call's records and every map equal the oracle's once the queue drains."""
    _gpu()
    from cilium_amd.datapath import Datapath, DeviceBatch, ING_OUT, to_numpy
    sc = synth.config2(n_flows=160_000, n_pairs=16_000, n_ep=40, n_ids=512, n_l3=200, n_l4=400, n_wc=8,
                       n_cidr=32, ct_max=400_000)
    made = synth.conntrack_local(sc, every=every, max_entries=mx)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    q = (pk.n + 7) // 8
    parts = [pk.slice(k * q, min(pk.n, (k + 1) * q)) for k in range(8)]
    dbs = [DeviceBatch(p) for p in parts]
    torch.cuda.synchronize()
    outs = [dp.ingress(db, sc.now + k) for k, db in enumerate(dbs)]
    torch.cuda.synchronize()
    for k, part in enumerate(parts):
        got, want = to_numpy(outs[k], ING_OUT), ref.ingress(part, sc.now + k)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, f"call {k}: {len(bad)} records differ, first {bad[:1]}"
    for name in made + ["cilium_ct4_global"]:
        assert dp.dump_map(name) == ref.dump(name), name
    # every local map evicted on every call (the oracle's log; the device's equal maps
    # say its evictions matched)
    assert all(len(ref.lru_log[n]) == 8 for n in made), {n: len(ref.lru_log[n]) for n in made}


@pytest.mark.gpu
def test_gpu_conntrack_local_batches_api():
    """gf_policy_ingress_classify_batches (schedules built on the aux stream) with
    per-endpoint maps: the same records and maps as the oracle."""
    _gpu()
    from cilium_amd.datapath import Datapath, DeviceBatch, ING_OUT, to_numpy
    sc = synth.fuzz(seed=5, n_packets=20000, n_batches=3)
    made = synth.conntrack_local(sc, every=2, max_entries=900)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    bs = [DeviceBatch(pk) for pk in sc.batches]
    outs = dp.ingress_batches(bs, [sc.now + k for k in range(len(bs))])
    torch.cuda.synchronize()
    for k, pk in enumerate(sc.batches):
        assert np.array_equal(to_numpy(outs[k], ING_OUT), ref.ingress(pk, sc.now + k)), f"batch {k}"
    for name in made + ["ct4", "ct6"]:
        assert dp.dump_map(name) == ref.dump(name), name


@pytest.mark.gpu
@pytest.mark.parametrize("seed,every,kw", [(5, 1, {"hazard": False}), (6, 2, {"hazard": True}),
                                           (11, 1, {"hazard": False, "icmp": False}), (12, 3, {"hazard": True})])
def test_gpu_conntrack_local_egress(seed, every, kw):
    """From-container (handle_ipv4_from_lxc / ipv6_l3_from_lxc on the sender's own
    CT_MAP4 / CT_MAP6, service entries included) and the local deliveries'
    handle_policy on the receiver's maps: records, rewritten frames, every CT map,
    policy counters and proxy maps equal the oracle's."""
    _gpu()
    from cilium_amd.datapath import Datapath, DeviceBatch, EG_OUT, to_numpy
    sc = synth.egress_fuzz(seed=seed, n_packets=20000, n_batches=3, **kw)
    made = synth.conntrack_local(sc, every=every)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        out, snap = dp.egress(DeviceBatch(pk, parse=False), sc.now + bi)
        torch.cuda.synchronize()
        ro, rs = ref.egress(pk, sc.now + bi)
        got = to_numpy(out, EG_OUT)
        bad = np.nonzero(got != ro)[0]
        assert len(bad) == 0, f"egress b{bi}: {len(bad)} records differ, first {bad[:1]}"
        assert not (snap.cpu().numpy() != rs).any(), f"frames b{bi}"
    for name in made + ["ct4", "ct6"]:
        assert dp.dump_map(name) == ref.dump(name), name
    grown = [n for n in made if n.startswith("ct4_") and len(ref.dump(n))]
    assert grown, "the senders' own maps should hold their connections"
    for e in range(16):
        assert dp.dump_map(f"pol{e}") == ref.dump(f"pol{e}"), f"pol{e}"
    assert dp.dump_map("cilium_proxy4") == ref.dump("cilium_proxy4")
    assert dp.dump_map("cilium_proxy6") == ref.dump("cilium_proxy6")
