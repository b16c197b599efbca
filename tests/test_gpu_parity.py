"""GPU parity: libgpuflow's HIP kernels vs the CPU oracle on the same seeded
inputs (bit-exact — integer/byte work).  Calls go through the C ABI."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from cilium_amd import synth
from cilium_amd.datapath import Datapath, DeviceBatch, LB_OUT, ING_OUT, PIPE_OUT, to_numpy
from oracle.scenario import OracleDP
import oracle.oracle as O


@pytest.fixture(scope="module", autouse=True)
def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _cmp_struct(a, b, what):
    if not np.array_equal(a, b):
        bad = np.nonzero(a != b)[0]
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} mismatches, first at {i}: gpu={a[i]} ref={b[i]}")


def test_parse_columns_match_oracle():
    sc = synth.fuzz(seed=11, n_packets=20000, n_batches=1)
    pk = sc.batches[0]
    b = DeviceBatch(pk)
    got = b.columns_numpy()
    ref = OracleDP(sc).parse(pk)
    for k in ("ethertype", "saddr4", "daddr4", "proto", "l4_off", "l4w0", "l4w3", "saddr6", "daddr6"):
        assert np.array_equal(got[k], ref[k]), k


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_all_programs(seed):
    sc = synth.fuzz(seed=seed, n_packets=20000, n_batches=3)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        b = DeviceBatch(pk)
        v, (lo, nd6), io = dp.xdp(b), dp.lb(b), dp.ingress(b, sc.now + bi)
        torch.cuda.synchronize()
        _cmp_struct(v.cpu().numpy(), ref.xdp(pk), f"xdp b{bi}")
        rl, rn6 = ref.lb(pk)
        _cmp_struct(to_numpy(lo, LB_OUT), rl, f"lb b{bi}")
        assert np.array_equal(nd6.cpu().numpy(), rn6), f"lb nd6 b{bi}"
        _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(pk, sc.now + bi), f"ingress b{bi}")
    # device-authoritative state pulled back through the map API
    assert dp.dump_map("ct4") == ref.dump("ct4")
    assert dp.dump_map("ct6") == ref.dump("ct6")
    for e in range(16):
        assert dp.dump_map(f"pol{e}") == ref.dump(f"pol{e}"), f"policy counters pol{e}"


@pytest.mark.parametrize("n_fix", [2_000, 6_000])
def test_config1_xdp_scaled(n_fix):
    """6,000 /32s do not fit the compact address set (<= 4,096 addresses): the /32
    probes take the hash table."""
    sc = synth.config1(n_packets=200_000, n_lpm=10_000, n_fix=n_fix, n_ep=1024)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    v = dp.xdp(DeviceBatch(pk))
    torch.cuda.synchronize()
    r = ref.xdp(pk)
    _cmp_struct(v.cpu().numpy(), r, "config1 xdp")
    assert 0.05 < (r == 1).mean() < 0.95


def test_xdp_address_sets_edge_keys():
    """k_xdp_lds's compact address sets (the /32 hash and cilium_lxc's IPv4 keys in
    LDS): address 0 in both (its own flag), a /32 map key whose prefixlen is not 32
    (never matched: the lookup key is {32, saddr}), and a map update between two
    calls (the set is rebuilt) — verdicts equal the oracle's."""
    from cilium_amd import bpf
    sc = synth.config1(n_packets=20_000, n_lpm=2_000, n_fix=500, n_ep=256)
    rng = np.random.default_rng(5)
    x = np.uint32(synth.ip4("198.51.100.7"))
    sc.maps["cilium_cidr_v4_fix"].keys = np.concatenate(
        [sc.maps["cilium_cidr_v4_fix"].keys, synth.lpm4_keys([32, 24], np.array([0, x], np.uint32))])
    sc.maps["cilium_cidr_v4_fix"].vals = np.concatenate([sc.maps["cilium_cidr_v4_fix"].vals, np.ones((2, 1), np.uint8)])
    lx = sc.maps["cilium_lxc"]
    lx.keys = np.concatenate([lx.keys, synth.endpoint_keys4(np.array([0], np.uint32))])
    lx.vals = np.concatenate([lx.vals, lx.vals[:1]])
    pk = sc.batches[0]
    n = pk.n
    ipv4 = (pk.frames[:, 12] == 8) & (pk.frames[:, 13] == 0) & (pk.lens >= 34)
    rows = np.nonzero(ipv4)[0]
    pick = rng.choice(rows, 600, replace=False)
    ep0 = synth.be32_bytes([0])[0]
    pk.frames[pick[:200], 26:30] = ep0                              # saddr 0.0.0.0: in the /32 set
    pk.frames[pick[200:400], 30:34] = ep0                           # daddr 0.0.0.0: an endpoint
    pk.frames[pick[400:], 26:30] = synth.be32_bytes([x])[0]         # only a /24 key holds x
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    v = dp.xdp(DeviceBatch(pk))
    torch.cuda.synchronize()
    r = ref.xdp(pk)
    _cmp_struct(v.cpu().numpy(), r, "xdp edge keys")
    assert (r[pick[:200]] == 1).all()
    # a /32 for x through the map API: the next call sees it
    k = synth.lpm4_keys([32], np.array([x], np.uint32))[0]
    bpf.UpdateElement(dp.fd["cilium_cidr_v4_fix"], k.tobytes(), bytes([1]))
    ref.m["cilium_cidr_v4_fix"].update(k.tobytes(), bytes([1]))
    v = dp.xdp(DeviceBatch(pk))
    torch.cuda.synchronize()
    r2 = ref.xdp(pk)
    _cmp_struct(v.cpu().numpy(), r2, "xdp after update")
    assert (r2[pick[400:]] == 1).all()


def test_xdp_dir24_tables_match_oracle(monkeypatch):
    """GF_XDP_DIR24=1: the v4 prefixes as DIR-24-8 tables (Map::dir24) in place of
    the trie walk, on config 1's prefix mix plus a /26 inside a covered /24, a /29
    and a /31 sharing one /24 group, and a prefix added through the map API
    between two calls (the tables rebuild after the trie) — verdicts equal the
    oracle's, through k_xdp_lds and the pipeline's k_xdp path alike."""
    from cilium_amd import bpf
    monkeypatch.setenv("GF_XDP_DIR24", "1")
    sc = synth.config1(n_packets=100_000, n_lpm=10_000, n_fix=2_000, n_ep=1024)
    lp = sc.maps["cilium_cidr_v4_dyn"]
    base = np.uint32(synth.ip4("203.0.113.0"))
    extra = synth.lpm4_keys([24, 26, 29, 31], np.array([base, base + 64, synth.ip4("198.18.7.8"),
                                                          synth.ip4("198.18.7.250")], np.uint32))
    lp.keys = np.concatenate([lp.keys, extra])
    lp.vals = np.concatenate([lp.vals, np.ones((len(extra), lp.vals.shape[1]), lp.vals.dtype)])
    pk = sc.batches[0]
    ipv4 = np.nonzero((pk.frames[:, 12] == 8) & (pk.frames[:, 13] == 0) & (pk.lens >= 34))[0]
    rng = np.random.default_rng(9)
    pick = rng.choice(ipv4, 1024, replace=False)
    probes = np.array([synth.ip4(a) for a in ("198.18.7.8", "198.18.7.15", "198.18.7.16", "198.18.7.250",
                                              "198.18.7.251", "198.18.7.252", "203.0.113.200", "198.18.8.1")],
                      np.uint32)
    pk.frames[pick, 26:30] = synth.be32_bytes(probes[np.arange(len(pick)) % len(probes)])
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    v = dp.xdp(DeviceBatch(pk))
    torch.cuda.synchronize()
    r = ref.xdp(pk)
    _cmp_struct(v.cpu().numpy(), r, "xdp dir24")
    k = synth.lpm4_keys([28], np.array([synth.ip4("198.18.8.0")], np.uint32))[0]
    bpf.UpdateElement(dp.fd["cilium_cidr_v4_dyn"], k.tobytes(), bytes(lp.vals.shape[1]))
    ref.m["cilium_cidr_v4_dyn"].update(k.tobytes(), bytes(lp.vals.shape[1]))
    v = dp.xdp(DeviceBatch(pk))
    torch.cuda.synchronize()
    r2 = ref.xdp(pk)
    _cmp_struct(v.cpu().numpy(), r2, "xdp dir24 after update")
    assert (r2[pick[np.arange(len(pick)) % len(probes) == 7]] == 1).all()     # 198.18.8.1: now under the /28


def test_config3_lb_scaled():
    sc = synth.config3(n_packets=200_000, n_svc=5_000)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    lo, _ = dp.lb(DeviceBatch(pk))
    torch.cuda.synchronize()
    rl, _ = ref.lb(pk)
    _cmp_struct(to_numpy(lo, LB_OUT), rl, "config3 lb")
    assert (rl["slave"] > 0).mean() > 0.5


def test_config2_ingress_scaled():
    sc = synth.config2(n_flows=60_000, n_pairs=8_000, n_ep=32, n_ids=512, n_l3=200, n_l4=400, n_wc=8,
                       n_cidr=32, ct_max=400_000)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        io = dp.ingress(DeviceBatch(pk), sc.now)
        torch.cuda.synchronize()
        _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(pk, sc.now), f"config2 batch {bi}")
    assert dp.dump_map("cilium_ct4_global") == ref.dump("cilium_ct4_global")


@pytest.mark.parametrize("n_pairs,n_flows", [(3, 2_500), (40, 6_000)])
def test_ingress_elephant_groups(n_pairs, n_flows):
    """Flow groups of thousands of packets in one batch (3 address pairs: buckets of
    ~3,300 packets, one lane each; 40 pairs: ~600) mixed with per-packet buckets
    (truncated / unknown-protocol packets): records and the CT equal the oracle's."""
    sc = synth.config2(n_flows=n_flows, n_pairs=n_pairs, n_ep=min(n_pairs, 8), n_ids=64, n_l3=40, n_l4=80, n_wc=8,
                       n_cidr=16, ct_max=200_000)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        io = dp.ingress(DeviceBatch(pk), sc.now + bi)
        torch.cuda.synchronize()
        _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(pk, sc.now + bi), f"elephants batch {bi}")
    assert dp.dump_map("cilium_ct4_global") == ref.dump("cilium_ct4_global")


def test_ingress_batches_pipelined_equals_oracle():
    """gf_policy_ingress_classify_batches (schedule of batch k+1 on a second stream
    while batch k runs) over the scaled config-2 stream and its fuzz sibling:
    every record of every batch and the CT afterwards equal the oracle's
    sequential batches."""
    for sc in (synth.config2(n_flows=60_000, n_pairs=8_000, n_ep=32, n_ids=512, n_l3=200, n_l4=400, n_wc=8,
                             n_cidr=32, ct_max=400_000), synth.fuzz(11, n_batches=4)):
        dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
        bs = [DeviceBatch(pk) for pk in sc.batches]
        nows = [sc.now + 3 * k for k in range(len(bs))]
        outs = dp.ingress_batches(bs, nows)
        torch.cuda.synchronize()
        for bi, (pk, io) in enumerate(zip(sc.batches, outs)):
            _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(pk, nows[bi]), f"{sc.name} batch {bi}")
        for name in sc.maps:
            if sc.maps[name].ksz in (14, 40):
                assert dp.dump_map(name) == ref.dump(name), name


def test_ingress_large_batch_properties():
    """Full-size-style property checks without the oracle: replaying the same
    established stream twice is idempotent for the verdict of REPLY packets and
    every packet gets exactly one record."""
    sc = synth.config2(n_flows=400_000, n_pairs=50_000, n_ep=64, n_ids=1024, n_l3=500, n_l4=1000, n_wc=8,
                       n_cidr=32, ct_max=2_000_000)
    dp = Datapath(sc, pin_prefix=None)
    outs = []
    for pk in sc.batches:
        io = dp.ingress(DeviceBatch(pk), sc.now)
        torch.cuda.synchronize()
        outs.append(to_numpy(io, ING_OUT))
    o = outs[-1]
    assert np.all(np.isin(o["action"], [0, 2, 7]))
    assert np.all((o["reason"] == 0) == (o["action"] != 2))


def test_ct_counter_carry_and_codec():
    """CT values live on the device in the GF_VCODEC_CT hot-split layout with the
    rx counters' low halves next to the key: entries whose rx_packets/rx_bytes sit
    at a 32-bit boundary must carry into the high halves exactly like the
    reference's u64 adds (conntrack.h:99-108), and lookups through the map API
    must decode to the reference ct_entry layout."""
    import struct
    from cilium_amd.synth import ip4, raw16, TCP
    E, R, NOW = ip4("10.1.0.5"), ip4("100.64.1.9"), 7000
    htonl = lambda x: struct.unpack("<I", struct.pack(">I", x))[0]
    sc = synth.Scenario("carry", now=NOW)
    # forward tuples (reversed at ingress: daddr=R, saddr=E... as ct_lookup4 leaves them), TUPLE_F_IN
    keys, vals = [], []
    for j, (rx, rxb) in enumerate([(0xffffffff, 100), (5, 0xfffffff0), (0xffffffff, 0xffffffff), (2**40 + 7, 2**33)]):
        k = struct.pack("<IIHHBB", htonl(R), htonl(E), raw16(8080 + j), raw16(40000), TCP, 1)
        v = struct.pack("<QQQQIHHHHI", rx, rxb, 11, 22, NOW + 100, 16, 0, 0, 0, 300)
        keys.append(np.frombuffer(k, np.uint8)); vals.append(np.frombuffer(v, np.uint8))
    sc.add_map(synth.MapSpec("ct4", synth.LRU_HASH, 14, 48, 1000, 0, np.stack(keys), np.stack(vals)))
    sc.add_map(synth.MapSpec("pol", synth.HASH, 8, 24, 16384, 0, synth.policy_keys([300], [0], [0]),
                             synth.policy_vals([0])))
    sc.lxc.append({"lxc_id": 7, "seclabel": 500, "policy": "pol", "ct4": "ct4", "ct6": None, "cidr4": None,
                   "cidr6": None, "revnat4": None, "revnat6": None, "flags": synth.LXC_PRODUCTION, "l4": []})
    n = 4
    f, l = synth.frames_v4(n, 64, [R] * n, [E] * n, [TCP] * n, [40000] * n, [8080 + j for j in range(n)],
                           [synth.F_ACK] * n, [8] * n, payload=10)
    l = np.array([40, 0x20, 0x30, 60], np.uint32) + 54
    pk = synth.Packets(f, l, np.full(n, 300, np.uint32), np.full(n, 42, np.uint32), np.full(n, 7, np.uint16),
                       np.zeros(n, np.uint8))
    sc.batches.append(pk)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    io = dp.ingress(DeviceBatch(pk), NOW)
    torch.cuda.synchronize()
    _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(pk, NOW), "ingress")
    got, want = dp.dump_map("ct4"), ref.dump("ct4")
    assert got == want
    rx = sorted(struct.unpack("<QQ", v[:16]) for v in got.values())
    assert (0x100000000, 100 + 94) in rx and (6, 0xfffffff0 + 0x20 + 54) in rx


@pytest.mark.parametrize("seed,kw", [(3, {}), (4, {"fixed_secctx": 300}), (8, {"lb_redirect": True}),
                                     (9, {"proxy_max": 12})])
def test_pipeline_fuzz(seed, kw):
    """Config 4 composition: bpf_xdp -> bpf_lb -> bpf_netdev -> handle_policy over
    raw frames; records, LB v6 addresses, the rewritten headers (MACs, TTL, daddr,
    ports, IPv4/L4 checksums) and the CT / policy state all bit-exact."""
    sc = synth.pipeline_fuzz(seed=seed, n_packets=20000, n_batches=3, **kw)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        b = DeviceBatch(pk, parse=False)
        out, nd6, snap = dp.pipeline(b, sc.now + bi)
        torch.cuda.synchronize()
        ro, rn6, rs = ref.pipeline(pk, sc.now + bi)
        _cmp_struct(to_numpy(out, PIPE_OUT), ro, f"pipeline b{bi}")
        assert np.array_equal(nd6.cpu().numpy(), rn6), f"pipeline nd6 b{bi}"
        got = snap.cpu().numpy()
        bad = np.nonzero((got != rs).any(axis=1))[0]
        assert len(bad) == 0, f"rewritten frames b{bi}: {len(bad)} rows differ, first {bad[:1]}"
        assert set(np.unique(ro["stage"])) >= {1, 3, 4}
    assert dp.dump_map("ct4") == ref.dump("ct4")
    assert dp.dump_map("ct6") == ref.dump("ct6")
    for e in range(16):
        assert dp.dump_map(f"pol{e}") == ref.dump(f"pol{e}"), f"policy counters pol{e}"
    # cilium_proxy4/6 entries of the proxy redirects (lib/lxc.h:96-205), batch-order semantics
    p4, p6 = ref.dump("cilium_proxy4"), ref.dump("cilium_proxy6")
    assert len(p4) > 0
    assert dp.dump_map("cilium_proxy4") == p4
    assert dp.dump_map("cilium_proxy6") == p6


def test_pipeline_dir24_prefilter(monkeypatch):
    """GF_XDP_DIR24=1 through the pipeline's front (k_pipe_front -> xdp_verdict): the
    fuzz pipeline with 400 more v4_dyn prefixes (/22-/31, a 16-bit trie root, so the
    DIR-24-8 tables are read) — records, rewritten frames and CT equal the oracle's."""
    monkeypatch.setenv("GF_XDP_DIR24", "1")
    sc = synth.pipeline_fuzz(seed=5, n_packets=20000, n_batches=2)
    rng = np.random.default_rng(21)
    pl = rng.integers(22, 32, 400).astype(np.uint32)
    nets = (np.uint32(synth.ip4("100.64.0.0")) + rng.integers(0, 1 << 18, 400).astype(np.uint32)) & \
        (~((np.uint32(1) << (32 - pl)) - np.uint32(1))).astype(np.uint32)
    m = sc.maps["v4_dyn"]
    keys = np.concatenate([m.keys, synth.lpm4_keys(pl, nets)])
    vals = np.concatenate([m.vals, np.ones((len(pl), m.vals.shape[1]), m.vals.dtype)])
    _, first = np.unique(keys, axis=0, return_index=True)
    m.keys, m.vals = keys[np.sort(first)], vals[np.sort(first)]
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        b = DeviceBatch(pk, parse=False)
        out, nd6, snap = dp.pipeline(b, sc.now + bi)
        torch.cuda.synchronize()
        ro, rn6, rs = ref.pipeline(pk, sc.now + bi)
        _cmp_struct(to_numpy(out, PIPE_OUT), ro, f"pipeline dir24 b{bi}")
        assert np.array_equal(snap.cpu().numpy(), rs), f"rewritten frames b{bi}"
        assert (ro["stage"] == 1).any()
    assert dp.dump_map("ct4") == ref.dump("ct4")


def test_pipeline_checksum_rewrites():
    """Frames with valid checksums through LB translations and port maps: the
    device rewrites equal the oracle's (which keep the checksums valid)."""
    from test_pipeline_oracle import _scenario
    sc = _scenario(n=4000, seed=12)
    pk = sc.batches[0]
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    out, nd6, snap = dp.pipeline(DeviceBatch(pk, parse=False), sc.now)
    torch.cuda.synchronize()
    ro, rn6, rs = ref.pipeline(pk, sc.now)
    _cmp_struct(to_numpy(out, PIPE_OUT), ro, "pipeline")
    assert np.array_equal(snap.cpu().numpy(), rs)


def test_ct_gc_device_sweep_then_traffic():
    """ctmap.GC on the device replica (expired entries and ct_delete tombstones
    removed, probe clusters compacted) equals the oracle's doGC4/doGC6, and the
    traffic after it still sees exactly the reference's CT state."""
    import ctypes as C
    from cilium_amd._lib import lib
    sc = synth.fuzz(seed=5, n_packets=20000, n_batches=4)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(bi, now):
        pk = sc.batches[bi]
        io = dp.ingress(DeviceBatch(pk), now)
        torch.cuda.synchronize()
        _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(pk, now), f"ingress b{bi}")

    run(0, sc.now)
    run(1, sc.now + 1)
    for name in ("ct4", "ct6"):
        got = lib.gf_ct_gc(dp.fd[name], sc.now + 11, st)
        assert got == ref.ct_gc(name, sc.now + 11) and got > 0, name
        assert dp.dump_map(name) == ref.dump(name), name
    run(2, sc.now + 200)
    for name in ("ct4", "ct6"):
        got = lib.gf_ct_gc(dp.fd[name], sc.now + 301, st)
        assert got == ref.ct_gc(name, sc.now + 301), name
    run(3, sc.now + 400)
    for name in ("ct4", "ct6"):
        assert dp.dump_map(name) == ref.dump(name), name
    assert lib.gf_ct_gc(dp.fd["ct4"], 0xFFFFFFFF, st) == ref.ct_gc("ct4", 0xFFFFFFFF)
    assert dp.dump_map("ct4") == {} == ref.dump("ct4")


def test_drop_notify_events():
    """send_drop_notify records (bpf/lib/drop.h:47-107) appended to the device
    event ring in batch order, for the ingress program and the full pipeline,
    equal the oracle's, capture bytes included."""
    import ctypes as C
    from cilium_amd._lib import lib, gf_event_ring
    cap = 200000
    recs = torch.zeros((cap, 160), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    ring = gf_event_ring(recs.data_ptr(), cap, cnt.data_ptr())
    assert lib.gf_set_event_ring(C.byref(ring)) == 0
    try:
        sc = synth.fuzz(seed=2, n_packets=20000, n_batches=2)
        dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
        exp = []
        for bi, pk in enumerate(sc.batches):
            io = dp.ingress(DeviceBatch(pk), sc.now + bi)
            ro = ref.ingress(pk, sc.now + bi)
            torch.cuda.synchronize()
            _cmp_struct(to_numpy(io, ING_OUT), ro, f"ingress b{bi}")
            exp.append(ref.ingress_events(pk, ro))
        e = np.concatenate(exp)
        n = int(cnt.item())
        assert n == len(e) > 100
        assert np.array_equal(recs[:n].cpu().numpy(), e)
        cnt.zero_()
        sc = synth.pipeline_fuzz(seed=3, n_packets=20000, n_batches=2)
        dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
        exp = []
        for bi, pk in enumerate(sc.batches):
            out, nd6, snap = dp.pipeline(DeviceBatch(pk, parse=False), sc.now + bi)
            ro, rn6, rs, ev = ref.pipeline(pk, sc.now + bi, events=True)
            torch.cuda.synchronize()
            _cmp_struct(to_numpy(out, PIPE_OUT), ro, f"pipeline b{bi}")
            exp.append(ev)
        e = np.concatenate(exp)
        n = int(cnt.item())
        assert n == len(e) > 100
        got = recs[:n].cpu().numpy()
        bad = np.nonzero((got != e).any(axis=1))[0]
        assert len(bad) == 0, f"{len(bad)} event records differ, first {bad[:1]}: {got[bad[0]][:32]} vs {e[bad[0]][:32]}"
        cnt.zero_()
        # endpoint egress: the sender's drops and the local deliveries' handle_policy drops
        from cilium_amd.datapath import EG_OUT
        sc = synth.egress_fuzz(seed=5, n_packets=20000, n_batches=2, hazard=False)
        dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
        exp = []
        for bi, pk in enumerate(sc.batches):
            out, snap = dp.egress(DeviceBatch(pk, parse=False), sc.now + bi)
            ro, rs, ev = ref.egress(pk, sc.now + bi, events=True)
            torch.cuda.synchronize()
            _cmp_struct(to_numpy(out, EG_OUT), ro, f"egress b{bi}")
            exp.append(ev)
        e = np.concatenate(exp)
        n = int(cnt.item())
        assert n == len(e) > 100
        got = recs[:n].cpu().numpy()
        bad = np.nonzero((got != e).any(axis=1))[0]
        assert len(bad) == 0, f"{len(bad)} egress event records differ, first {bad[:1]}: {got[bad[0]][:32]} vs {e[bad[0]][:32]}"
    finally:
        lib.gf_set_event_ring(None)


def _trace_on(sc, every=2, netdev_ifindex=None):
    """TRACE_NOTIFY on every `every`-th endpoint program (per-endpoint define,
    pkg/endpoint/endpoint.go:131-134) and, for a pipeline, on the netdev."""
    for k, e in enumerate(sc.lxc):
        if k % every == 0:
            e["flags"] |= synth.LXC_TRACE_NOTIFY
    if netdev_ifindex is not None and sc.netdev is not None:
        sc.netdev = dict(sc.netdev, flags=sc.netdev.get("flags", 0) | synth.NETDEV_TRACE_NOTIFY,
                         ingress_ifindex=netdev_ifindex)


def _ring_check(recs, cnt, e, what):
    n = int(cnt.item())
    assert n == len(e), f"{what}: {n} records vs {len(e)}"
    got = recs[:n].cpu().numpy()
    bad = np.nonzero((got != e).any(axis=1))[0]
    assert len(bad) == 0, f"{what}: {len(bad)} records differ, first {bad[:1]}: {got[bad[0]][:32]} vs {e[bad[0]][:32]}"
    return got


def test_trace_notify_events():
    """send_trace_notify records (bpf/lib/trace.h:59-106) interleaved with the drop
    records in the device event ring — per packet in the order the programs send
    them (from_netdev / handle_ingress first, the redirects' TO_PROXY with the frame
    before its rewrites, TO_HOST / TO_STACK / TO_OVERLAY / TO_LXC, the drop last) —
    equal the oracle's per-packet event lists, capture bytes included, for the
    ingress program, the full pipeline and endpoint egress; programs without
    TRACE_NOTIFY send none."""
    import ctypes as C
    from cilium_amd._lib import lib, gf_event_ring
    from cilium_amd.datapath import EG_OUT
    cap = 400000
    recs = torch.zeros((cap, 160), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    ring = gf_event_ring(recs.data_ptr(), cap, cnt.data_ptr())
    assert lib.gf_set_event_ring(C.byref(ring)) == 0
    try:
        sc = synth.fuzz(seed=2, n_packets=20000, n_batches=2)
        _trace_on(sc)
        dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
        exp = []
        for bi, pk in enumerate(sc.batches):
            io = dp.ingress(DeviceBatch(pk), sc.now + bi)
            with O.TraceSink(pk.n, capture=False) as ts:
                ro = ref.ingress(pk, sc.now + bi)
                ref.ingress_events(pk, ro)
            torch.cuda.synchronize()
            _cmp_struct(to_numpy(io, ING_OUT), ro, f"ingress b{bi}")
            exp.append(ts.events())
        got = _ring_check(recs, cnt, np.concatenate(exp), "ingress")
        assert (got[:, 0] == 4).sum() > 1000 and (got[:, 0] == 1).sum() > 100
        cnt.zero_()
        sc = synth.pipeline_fuzz(seed=3, n_packets=20000, n_batches=2)
        _trace_on(sc, every=3, netdev_ifindex=7)
        dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
        exp = []
        for bi, pk in enumerate(sc.batches):
            out, nd6, snap = dp.pipeline(DeviceBatch(pk, parse=False), sc.now + bi)
            with O.TraceSink(pk.n) as ts:
                ro, rn6, rs = ref.pipeline(pk, sc.now + bi)
            torch.cuda.synchronize()
            _cmp_struct(to_numpy(out, PIPE_OUT), ro, f"pipeline b{bi}")
            exp.append(ts.events())
        got = _ring_check(recs, cnt, np.concatenate(exp), "pipeline")
        assert set(np.unique(got[got[:, 0] == 4, 1])) >= {0, 8}
        cnt.zero_()
        for seed, kw in ((5, {"hazard": False}), (6, {"hazard": True})):
            sc = synth.egress_fuzz(seed=seed, n_packets=20000, n_batches=2, **kw)
            _trace_on(sc)
            dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
            exp = []
            for bi, pk in enumerate(sc.batches):
                out, snap = dp.egress(DeviceBatch(pk, parse=False), sc.now + bi)
                with O.TraceSink(pk.n) as ts:
                    ro, rs = ref.egress(pk, sc.now + bi)
                torch.cuda.synchronize()
                _cmp_struct(to_numpy(out, EG_OUT), ro, f"egress s{seed} b{bi}")
                exp.append(ts.events())
            got = _ring_check(recs, cnt, np.concatenate(exp), f"egress s{seed}")
            assert set(np.unique(got[got[:, 0] == 4, 1])) >= {0, 1, 3, 4, 5}, np.unique(got[got[:, 0] == 4, 1])
            cnt.zero_()
    finally:
        lib.gf_set_event_ring(None)


@pytest.mark.parametrize("seed,kw", [(5, {"hazard": False}), (6, {"hazard": True}),
                                     (7, {"hazard": False, "proxy_max": 6}),
                                     (11, {"hazard": False, "icmp": False}), (12, {"hazard": True, "icmp": False})])
def test_egress_fuzz(seed, kw):
    """Endpoint egress (bpf_lxc.c handle_ingress -> handle_ipv4_from_lxc /
    ipv6_l3_from_lxc) over raw frames, local deliveries through the destination's
    handle_policy: records, rewritten frames, CT v4/v6 (service / loopback /
    related entries, tx accounting, deletes), policy counters and the proxy maps
    all bit-exact vs the oracle."""
    from cilium_amd.datapath import EG_OUT
    sc = synth.egress_fuzz(seed=seed, n_packets=20000, n_batches=3, **kw)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        b = DeviceBatch(pk, parse=False)
        out, snap = dp.egress(b, sc.now + bi)
        torch.cuda.synchronize()
        ro, rs = ref.egress(pk, sc.now + bi)
        _cmp_struct(to_numpy(out, EG_OUT), ro, f"egress b{bi}")
        got = snap.cpu().numpy()
        bad = np.nonzero((got != rs).any(axis=1))[0]
        assert len(bad) == 0, f"rewritten frames b{bi}: {len(bad)} rows differ, first {bad[:1]}"
        assert set(np.unique(ro["stage"])) >= {0, 4, 5}
    assert dp.dump_map("ct4") == ref.dump("ct4")
    assert dp.dump_map("ct6") == ref.dump("ct6")
    for e in range(16):
        assert dp.dump_map(f"pol{e}") == ref.dump(f"pol{e}"), f"policy counters pol{e}"
    assert dp.dump_map("cilium_proxy4") == ref.dump("cilium_proxy4")
    assert dp.dump_map("cilium_proxy6") == ref.dump("cilium_proxy6")


def test_pipeline_partition_owners():
    """gf_pipeline_partition (ingest re-partition for N GPUs): the owner of every
    frame is its flow group's rank after bpf_lb's translation, as the host
    restatement computes it from the oracle's LB results; stable owner order and
    per-rank counts."""
    from cilium_amd import shard
    from oracle.parity import owners_host
    sc = synth.pipeline_fuzz(seed=22, n_packets=20000, n_batches=2)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for world, rank in ((2, 1), (3, 0), (8, 5)):
        for pk in sc.batches:
            b = DeviceBatch(pk, parse=False)
            owner, order, counts = shard.partition(dp, b.frames, b.len, rank, world, b.flow_hash, b.tc_index)
            lo, nd6 = ref.lb(pk)
            want = owners_host(lo, nd6, pk, rank, world)
            assert np.array_equal(owner.cpu().numpy(), want)
            assert np.array_equal(order.cpu().numpy(), np.argsort(want, kind="stable"))
            assert np.array_equal(counts.cpu().numpy(), np.bincount(want, minlength=world))


def test_stream_counter_block():
    """k_xdp / k_lb's wave-aggregated counter block (the block bench.py reads and
    the multi-GPU all-reduce sums): reason / action bins, packets and wire bytes
    equal the histogram of the oracle's verdicts, over a grid-stride launch with
    a ragged tail."""
    import ctypes as C
    from cilium_amd._lib import lib
    sc = synth.config3(n_packets=300_001, n_svc=5_000)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    lens = np.asarray(pk.lens, dtype=np.int64)
    cnt = torch.zeros(512, dtype=torch.int64, device="cuda")
    lib.gf_set_stats_sink(C.c_void_p(cnt.data_ptr()))
    try:
        lo, _ = dp.lb(DeviceBatch(pk))
        torch.cuda.synchronize()
    finally:
        lib.gf_set_stats_sink(None)
    c = cnt.cpu().numpy()
    rl, _ = ref.lb(pk)
    _cmp_struct(to_numpy(lo, LB_OUT), rl, "config3 lb")
    assert c[268] == pk.n and c[269] == lens.sum()
    for a in np.unique(rl["action"]):
        assert c[256 + int(a)] == (rl["action"] == a).sum(), f"action {a}"
    for r in range(1, 256):
        assert c[r] == (rl["reason"] == r).sum(), f"reason {r}"

    sc = synth.config1(n_packets=100_003, n_lpm=2_000, n_fix=500, n_ep=256)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    cnt.zero_()
    lib.gf_set_stats_sink(C.c_void_p(cnt.data_ptr()))
    try:
        dp.xdp(DeviceBatch(pk))
        torch.cuda.synchronize()
    finally:
        lib.gf_set_stats_sink(None)
    c = cnt.cpu().numpy()
    r = ref.xdp(pk)
    assert c[268] == pk.n and c[269] == np.asarray(pk.lens, dtype=np.int64).sum()
    assert c[257] == c[1] == (r == 1).sum() and c[258] == (r == 2).sum()


def test_stream_kernels_grid_stride(monkeypatch):
    """k_xdp and k_lb with the grid capped at 3 blocks (every block runs many
    tiles of its grid-stride loop, the last one ragged) stay bit-exact; the
    pipeline (k_pipe_front's wave-aggregated counters, one tile per block) on a
    ragged batch too, rewritten frames included."""
    monkeypatch.setenv("GPUFLOW_STREAM_GRID", "3")
    sc = synth.fuzz(seed=11, n_packets=5_003, n_batches=1)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk = sc.batches[0]
    b = DeviceBatch(pk)
    v, (lo, nd6) = dp.xdp(b), dp.lb(b)
    torch.cuda.synchronize()
    _cmp_struct(v.cpu().numpy(), ref.xdp(pk), "xdp")
    rl, rn6 = ref.lb(pk)
    _cmp_struct(to_numpy(lo, LB_OUT), rl, "lb")
    assert np.array_equal(nd6.cpu().numpy(), rn6)
    sc = synth.pipeline_fuzz(seed=12, n_packets=5_003, n_batches=2)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        out, nd6, snap = dp.pipeline(DeviceBatch(pk, parse=False), sc.now + bi)
        torch.cuda.synchronize()
        ro, rn6, rs = ref.pipeline(pk, sc.now + bi)
        _cmp_struct(to_numpy(out, PIPE_OUT), ro, f"pipeline b{bi}")
        assert np.array_equal(snap.cpu().numpy(), rs), f"rewritten frames b{bi}"
        assert np.array_equal(nd6.cpu().numpy(), rn6), f"pipeline nd6 b{bi}"


def test_ingress_counter_block():
    """k_ing_groups' counter block (reason / action bins shared, byte sums and
    CT-result counts kept per lane and folded at the end) equals the histogram
    of the oracle's handle_policy outputs."""
    import ctypes as C
    from cilium_amd._lib import lib
    sc = synth.fuzz(seed=13, n_packets=30_001, n_batches=2)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    cnt = torch.zeros(512, dtype=torch.int64, device="cuda")
    want = np.zeros(512, dtype=np.int64)
    for bi, pk in enumerate(sc.batches):
        b = DeviceBatch(pk)
        lib.gf_set_stats_sink(C.c_void_p(cnt.data_ptr()))
        try:
            io = dp.ingress(b, sc.now + bi)
            torch.cuda.synchronize()
        finally:
            lib.gf_set_stats_sink(None)
        ro = ref.ingress(pk, sc.now + bi)
        _cmp_struct(to_numpy(io, ING_OUT), ro, f"ingress b{bi}")
        np.add.at(want, ro["reason"].astype(np.int64), 1)
        np.add.at(want, 256 + ro["action"].astype(np.int64), 1)
        np.add.at(want, 264 + (ro["ct_ret"].astype(np.int64) & 3), 1)
        want[268] += pk.n
        want[269] += np.asarray(pk.lens, dtype=np.int64).sum()
    c = cnt.cpu().numpy()
    assert np.array_equal(c[:270], want[:270]), np.nonzero(c[:270] != want[:270])
    assert c[270] > 0


def test_egress_counter_block():
    """The endpoint-egress leg's counter block (k_eg_front wave-aggregated,
    k_eg_groups per-lane sums, local deliveries counted by handle_policy): one
    count per packet in its final reason / action bin, packets and wire bytes."""
    import ctypes as C
    from cilium_amd._lib import lib
    from cilium_amd.datapath import EG_OUT
    sc = synth.egress_fuzz(seed=8, n_packets=20001, n_batches=2, hazard=False)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    cnt = torch.zeros(512, dtype=torch.int64, device="cuda")
    want = np.zeros(512, dtype=np.int64)
    for bi, pk in enumerate(sc.batches):
        lib.gf_set_stats_sink(C.c_void_p(cnt.data_ptr()))
        try:
            out, _ = dp.egress(DeviceBatch(pk, parse=False), sc.now + bi)
            torch.cuda.synchronize()
        finally:
            lib.gf_set_stats_sink(None)
        ro, _ = ref.egress(pk, sc.now + bi)
        _cmp_struct(to_numpy(out, EG_OUT), ro, f"egress b{bi}")
        np.add.at(want, ro["reason"].astype(np.int64), 1)
        np.add.at(want, 256 + ro["action"].astype(np.int64), 1)
        want[268] += pk.n
        want[269] += np.asarray(pk.lens, dtype=np.int64).sum()
    c = cnt.cpu().numpy()
    assert c[268] == want[268] and c[269] == want[269]
    assert np.array_equal(c[:264], want[:264]), np.nonzero(c[:264] != want[:264])


RAGGED = (0, 1, 2, 63, 64, 65, 0, 4095, 4097, 1)


def test_empty_and_ragged_batches():
    """Batches of 0, 1, 2, one wave +-1 and one schedule tile +-1 packets, in
    sequence on one datapath (CT state carried from batch to batch): k_xdp /
    k_lb / handle_policy, the full pipeline and endpoint egress each equal the
    oracle; an empty batch is a no-op (return 0, nothing written, no state
    change) at every entry point, and the batched ingress call takes an empty
    batch between two others."""
    from cilium_amd.datapath import EG_OUT
    sc = synth.fuzz(seed=41, n_packets=20000, n_batches=1)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk, a = sc.batches[0], 0
    for i, n in enumerate(RAGGED):
        p = pk.slice(a, a + n)
        a += n
        b = DeviceBatch(p)
        v, (lo, nd6), io = dp.xdp(b), dp.lb(b), dp.ingress(b, sc.now + i)
        torch.cuda.synchronize()
        _cmp_struct(v.cpu().numpy(), ref.xdp(p), f"xdp n={n}")
        rl, rn6 = ref.lb(p)
        _cmp_struct(to_numpy(lo, LB_OUT), rl, f"lb n={n}")
        assert np.array_equal(nd6.cpu().numpy(), rn6), f"lb nd6 n={n}"
        _cmp_struct(to_numpy(io, ING_OUT), ref.ingress(p, sc.now + i), f"ingress n={n}")
    bs = [pk.slice(a, a + 3000), pk.slice(0, 0), pk.slice(a + 3000, a + 3001)]
    outs = dp.ingress_batches([DeviceBatch(p) for p in bs], [sc.now + 20 + k for k in range(3)])
    torch.cuda.synchronize()
    for k, p in enumerate(bs):
        _cmp_struct(to_numpy(outs[k], ING_OUT), ref.ingress(p, sc.now + 20 + k), f"ingress_batches {k}")
    assert dp.dump_map("ct4") == ref.dump("ct4")
    assert dp.dump_map("ct6") == ref.dump("ct6")

    sc = synth.pipeline_fuzz(seed=42, n_packets=20000, n_batches=1)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk, a = sc.batches[0], 0
    for i, n in enumerate(RAGGED):
        p = pk.slice(a, a + n)
        a += n
        out, nd6, snap = dp.pipeline(DeviceBatch(p, parse=False), sc.now + i)
        torch.cuda.synchronize()
        ro, rn6, rs = ref.pipeline(p, sc.now + i)
        _cmp_struct(to_numpy(out, PIPE_OUT), ro, f"pipeline n={n}")
        assert np.array_equal(nd6.cpu().numpy(), rn6), f"pipeline nd6 n={n}"
        assert np.array_equal(snap.cpu().numpy(), rs), f"pipeline frames n={n}"
    for m in ("ct4", "ct6"):
        assert dp.dump_map(m) == ref.dump(m), m

    sc = synth.egress_fuzz(seed=43, n_packets=20000, n_batches=1, hazard=True)
    dp, ref = Datapath(sc, pin_prefix=None), OracleDP(sc)
    pk, a = sc.batches[0], 0
    for i, n in enumerate(RAGGED):
        p = pk.slice(a, a + n)
        a += n
        out, snap = dp.egress(DeviceBatch(p, parse=False), sc.now + i)
        torch.cuda.synchronize()
        ro, rs = ref.egress(p, sc.now + i)
        _cmp_struct(to_numpy(out, EG_OUT), ro, f"egress n={n}")
        assert np.array_equal(snap.cpu().numpy(), rs), f"egress frames n={n}"
    for m in ("ct4", "ct6", "cilium_proxy4", "cilium_proxy6"):
        assert dp.dump_map(m) == ref.dump(m), m


def test_classify_argument_checks():
    """The classify calls' argument checks (the C ABI returns -errno the way the
    bpf(2) wrappers see the kernel, before anything is launched): a handle of the
    wrong kind is -EBADF, a missing column or output -EFAULT, a batch over 2^30
    packets -E2BIG, a frame stride too short for the headers -EINVAL; an empty
    batch is 0 with null pointers.  No failed call writes an output or changes the
    CT (gf_kernels.hip check_cols, gf_xdp_classify, gf_lb_classify,
    gf_policy_ingress_classify, gf_pipeline_classify, gf_lxc_egress_classify)."""
    import ctypes as C
    import errno
    from cilium_amd._lib import lib, gf_frames, gf_pkt_cols, gf_pipe_batch, gf_lxc_batch
    sc = synth.pipeline_fuzz(seed=44, n_packets=1000, n_batches=1)
    dp = Datapath(sc, pin_prefix=None)
    assert dp.xdp_prog and dp.lb_prog and dp.policy_array and dp.pipe
    b = DeviceBatch(sc.batches[0])
    torch.cuda.synchronize()
    n, stride = b.n, b.frames.shape[1]
    out = torch.full((n, 24), 0xAB, dtype=torch.uint8, device="cuda")
    nd6 = torch.full((n, 16), 0xAB, dtype=torch.uint8, device="cuda")
    o, d6 = out.data_ptr(), nd6.data_ptr()
    ct0 = dp.dump_map("ct4"), dp.dump_map("ct6")
    now = sc.now
    c = b.cols()

    def fr(k=n, st=stride, snap=b.frames.data_ptr(), ln=b.len.data_ptr()):
        return gf_frames(k, st, snap, ln)

    E = lambda e: -getattr(errno, e)
    # a handle of another kind, or none
    assert lib.gf_xdp_classify(dp.lb_prog, C.byref(c), o, None) == E("EBADF")
    assert lib.gf_lb_classify(dp.xdp_prog, C.byref(c), o, d6, None) == E("EBADF")
    assert lib.gf_policy_ingress_classify(dp.pipe, C.byref(c), now, o, None) == E("EBADF")
    assert lib.gf_pipeline_classify(dp.policy_array, C.byref(gf_pipe_batch(fr(), None, None)), now, o, d6, None,
                                    None) == E("EBADF")
    assert lib.gf_lxc_egress_classify(dp.xdp_prog, C.byref(gf_lxc_batch(fr(), None, None)), now, o, None,
                                      None) == E("EBADF")
    assert lib.gf_xdp_classify(987654, C.byref(c), o, None) == E("EBADF")
    # missing outputs / columns
    assert lib.gf_xdp_classify(dp.xdp_prog, C.byref(c), None, None) == E("EFAULT")
    assert lib.gf_lb_classify(dp.lb_prog, C.byref(c), None, d6, None) == E("EFAULT")
    assert lib.gf_policy_ingress_classify(dp.policy_array, C.byref(c), now, None, None) == E("EFAULT")
    assert lib.gf_policy_ingress_classify(dp.policy_array, None, now, o, None) == E("EFAULT")
    nc = b.cols()
    nc.saddr4 = None
    assert lib.gf_xdp_classify(dp.xdp_prog, C.byref(nc), o, None) == E("EFAULT")
    assert lib.gf_pipeline_classify(dp.pipe, C.byref(gf_pipe_batch(fr(ln=None), None, None)), now, o, d6, None,
                                    None) == E("EFAULT")
    assert lib.gf_lxc_egress_classify(dp.policy_array, C.byref(gf_lxc_batch(fr(snap=None), None, None)), now, o,
                                      None, None) == E("EFAULT")
    # too many packets for one call (checked before any launch reads the columns)
    big = b.cols()
    big.n = (1 << 30) + 1
    assert lib.gf_policy_ingress_classify(dp.policy_array, C.byref(big), now, o, None) == E("E2BIG")
    assert lib.gf_pipeline_classify(dp.pipe, C.byref(gf_pipe_batch(fr(k=(1 << 30) + 1), None, None)), now, o, d6,
                                    None, None) == E("E2BIG")
    assert lib.gf_lxc_egress_classify(dp.policy_array, C.byref(gf_lxc_batch(fr(k=(1 << 30) + 1), None, None)), now,
                                      o, None, None) == E("E2BIG")
    # a stride that cannot hold the headers the program parses
    assert lib.gf_pipeline_classify(dp.pipe, C.byref(gf_pipe_batch(fr(st=13), None, None)), now, o, d6, None,
                                    None) == E("EINVAL")
    assert lib.gf_lxc_egress_classify(dp.policy_array, C.byref(gf_lxc_batch(fr(st=33), None, None)), now, o, None,
                                      None) == E("EINVAL")
    # an empty batch: nothing to read or write
    z = gf_pkt_cols()
    z.n = 0
    assert lib.gf_xdp_classify(dp.xdp_prog, C.byref(z), None, None) == 0
    assert lib.gf_lb_classify(dp.lb_prog, C.byref(z), None, None, None) == 0
    assert lib.gf_policy_ingress_classify(dp.policy_array, C.byref(z), now, None, None) == 0
    assert lib.gf_pipeline_classify(dp.pipe, C.byref(gf_pipe_batch(gf_frames(0, 0, None, None), None, None)), now,
                                    None, None, None, None) == 0
    assert lib.gf_lxc_egress_classify(dp.policy_array, C.byref(gf_lxc_batch(gf_frames(0, 0, None, None), None, None)),
                                      now, None, None, None) == 0
    torch.cuda.synchronize()
    assert bool((out == 0xAB).all()) and bool((nd6 == 0xAB).all()), "a refused call wrote its output"
    assert (dp.dump_map("ct4"), dp.dump_map("ct6")) == ct0
    # and the program still classifies afterwards
    ref = OracleDP(sc)
    got, _, _ = dp.pipeline(DeviceBatch(sc.batches[0], parse=False), now)
    torch.cuda.synchronize()
    ro, _, _ = ref.pipeline(sc.batches[0], now)
    _cmp_struct(to_numpy(got, PIPE_OUT), ro, "pipeline after refused calls")
