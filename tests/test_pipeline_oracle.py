"""CPU checks of the full-pipeline oracle (bpf_xdp -> bpf_lb -> bpf_netdev ->
handle_policy, BASELINE config 4): the threaded restatement equals the
sequential one, and the header rewrites keep correct checksums correct — the
incremental-update arithmetic of bpf_l3_csum_replace / bpf_l4_csum_replace /
bpf_csum_diff (RFC 1624) checked against checksums recomputed from scratch."""
import numpy as np

from cilium_amd import synth
from cilium_amd.synth import ip4, TCP, UDP, ICMP, ICMPV6
from oracle.scenario import OracleDP


def test_pipeline_threads_equal_sequential():
    sc = synth.pipeline_fuzz(seed=5, n_packets=6000, n_batches=2)
    a, b = OracleDP(sc), OracleDP(sc, shards=4)
    for bi, pk in enumerate(sc.batches):
        o1, n1, s1 = a.pipeline(pk, sc.now + bi, threads=1)
        o2, n2, s2 = b.pipeline(pk, sc.now + bi, threads=4)
        assert np.array_equal(o1, o2) and np.array_equal(n1, n2) and np.array_equal(s1, s2)
    assert a.dump("ct4") == b.dump("ct4")
    for e in range(16):
        assert a.dump(f"pol{e}") == b.dump(f"pol{e}")
    assert a.dump("cilium_proxy4") == b.dump("cilium_proxy4") and len(a.dump("cilium_proxy4")) > 0


def test_proxy_map_full_is_sequential():
    """cilium_proxy4 updates in batch order: with a map that fills inside the
    batch, exactly the redirects past capacity become DROP_PROXYMAP_CREATE_FAILED
    (-161), sequential and threaded restatements alike."""
    sc = synth.pipeline_fuzz(seed=9, n_packets=20000, n_batches=2, proxy_max=12)
    a, b = OracleDP(sc), OracleDP(sc, shards=4)
    fails = 0
    for bi, pk in enumerate(sc.batches):
        o1, _, s1 = a.pipeline(pk, sc.now + bi, threads=1)
        o2, _, s2 = b.pipeline(pk, sc.now + bi, threads=4)
        assert np.array_equal(o1, o2) and np.array_equal(s1, s2)
        fails += int((o1["reason"] == 161).sum())
    assert fails > 0
    assert len(a.dump("cilium_proxy4")) == 12


def test_pipeline_stage_accounting():
    sc = synth.pipeline_fuzz(seed=6, n_packets=8000, n_batches=1)
    out, nd6, snap = OracleDP(sc).pipeline(sc.batches[0], sc.now)
    st = out["stage"]
    assert set(np.unique(st)) <= {1, 2, 3, 4}
    for s in (1, 3, 4):
        assert (st == s).sum() > 50, s
    assert np.all(out["action"][st == 1] == 1)                      # XDP_DROP
    assert np.all((out["reason"] == 0) == (out["action"] != 2))
    assert ((out["flags"] & 0x40) != 0).sum() > 50                  # LB translations reached netdev
    assert ((out["flags"] & 0x80) != 0).sum() > 20                  # port maps applied
    assert ((out["flags"] & 0x20) != 0).sum() > 0                   # ICMPv6 time exceeded
    assert np.all(out["lxc_id"][st != 4] == 0)


def _csum(b):
    b = bytes(b)
    if len(b) % 2:
        b += b"\0"
    s = sum(int.from_bytes(b[k:k + 2], "big") for k in range(0, len(b), 2))
    while s >> 16:
        s = (s & 0xffff) + (s >> 16)
    return s


def _scenario(n=3000, seed=9):
    """Frames with valid IPv4 header and TCP/UDP/ICMPv6 checksums through LB
    translations (with port rewrites, incl. the L3-fallback old-port-0 case)
    and endpoint delivery with port maps."""
    rng = np.random.default_rng(seed)
    sc = synth.Scenario("csum", now=100)
    n_ep = 8
    ep4 = (ip4("10.2.0.1") + np.arange(n_ep)).astype(np.uint32)
    ep6 = synth.rand_v6(rng, n_ep, prefix=(0xf0, 0x0d))
    vip4 = (ip4("10.97.0.1") + np.arange(4)).astype(np.uint32)
    vip6 = synth.rand_v6(rng, 4, prefix=(0xfd, 0x01))
    lk = np.concatenate([synth.endpoint_keys4(ep4), synth.endpoint_keys6(ep6)])
    lv = synth.endpoint_infos(np.arange(2 * n_ep) + 10, np.full(2 * n_ep, 300), np.full(2 * n_ep, 77),
                              np.zeros(2 * n_ep))
    lv[:, 16:22] = 0xaa
    lv[:, 24:30] = 0xbb
    for e in range(0, 2 * n_ep, 2):                                  # port maps 80 -> 8080, 53 -> 5353
        lv[e, 48:56] = np.array([synth.raw16(80), synth.raw16(8080), synth.raw16(53), synth.raw16(5353)],
                                "<u2").view(np.uint8)
    sc.add_map(synth.MapSpec("cilium_lxc", synth.HASH, 20, 112, 65535, 0, lk, lv))
    keys, vals = [], []
    for i, vip in enumerate(vip4):
        fp = [80, 53, 0, 443][i]
        keys.append(synth.lb4_keys([vip], [fp], [0])); vals.append(synth.lb4_vals([0], [0], [2], [0]))
        for s in (1, 2):
            keys.append(synth.lb4_keys([vip], [fp], [s]))
            vals.append(synth.lb4_vals([ep4[(i + s) % n_ep]], [[8443, 53, 9000, 0][i]], [0], [i + 1]))
    k4, v4 = synth.dedup(np.concatenate(keys), np.concatenate(vals))
    sc.add_map(synth.MapSpec("lb4", synth.HASH, 8, 12, 1024, 0, k4, v4))
    keys, vals = [], []
    for i in range(4):
        fp = [80, 53, 0, 443][i]
        keys.append(synth.lb6_keys(vip6[i:i + 1], [fp], [0]))
        vals.append(synth.lb6_vals(np.zeros((1, 16), np.uint8), [0], [2], [0]))
        for s in (1, 2):
            keys.append(synth.lb6_keys(vip6[i:i + 1], [fp], [s]))
            vals.append(synth.lb6_vals(ep6[(i + s) % n_ep][None, :], [[8443, 53, 9000, 0][i]], [0], [0]))
    k6, v6 = synth.dedup(np.concatenate(keys), np.concatenate(vals))
    sc.add_map(synth.MapSpec("lb6", synth.HASH, 20, 24, 1024, 0, k6, v6))
    sc.lb = {"lb4": "lb4", "lb6": "lb6", "flags": synth.LB_L3 | synth.LB_L4}
    sc.add_map(synth.MapSpec("pol", synth.HASH, 8, 24, 1024, 0, synth.policy_keys([2], [0], [0]),
                             synth.policy_vals([0])))
    sc.add_map(synth.MapSpec("ct4", synth.LRU_HASH, 14, 48, 100000))
    sc.add_map(synth.MapSpec("ct6", synth.LRU_HASH, 40, 48, 100000))
    sc.lxc.append({"lxc_id": 77, "seclabel": 300, "policy": "pol", "ct4": "ct4", "ct6": "ct6", "cidr4": None,
                   "cidr6": None, "revnat4": None, "revnat6": None, "flags": synth.LXC_PRODUCTION, "l4": []})
    sc.netdev = {"lxc_map": "cilium_lxc"}
    sc.meta["l3_only"] = (vip4[2], bytes(vip6[2]))
    stride = 128
    v6m = rng.random(n) < 0.4
    pr = rng.choice(np.array([TCP, UDP, ICMP], np.uint8), n)
    dports = np.array([80, 53, 443, 1234])[rng.integers(0, 4, n)]
    to_vip = rng.random(n) < 0.6
    d4 = np.where(to_vip, vip4[rng.integers(0, 4, n)], ep4[rng.integers(0, n_ep, n)])
    s4 = (ip4("192.0.2.0") + rng.integers(0, 256, n)).astype(np.uint32)
    f, lens = synth.frames_v4(n, stride, s4, d4, pr, rng.integers(1024, 65535, n), dports, synth.F_ACK, 8,
                              payload=rng.integers(0, 24, n))
    f[:, 34:stride] = np.where(np.arange(34, stride) < lens[:, None], f[:, 34:stride], 0)
    i6 = np.nonzero(v6m)[0]
    d6 = np.where(rng.random(len(i6))[:, None] < 0.6, vip6[rng.integers(0, 4, len(i6))], ep6[rng.integers(0, n_ep, len(i6))])
    s6 = synth.rand_v6(rng, len(i6))
    nh6 = np.where(pr[i6] == ICMP, ICMPV6, pr[i6]).astype(np.uint8)
    f6, l6 = synth.frames_v6(len(i6), stride, s6, d6, nh6, rng.integers(1024, 65535, len(i6)), dports[i6],
                             synth.F_ACK, 128, payload=rng.integers(0, 24, len(i6)))
    f[i6], lens[i6] = f6, l6
    for r in range(n):                                               # valid checksums
        fr, L = f[r], int(lens[r])
        if r in set(i6.tolist()):
            nh, l4 = int(fr[20]), 54
            pseudo = bytes(fr[22:54]) + (L - 54).to_bytes(4, "big") + bytes([0, 0, 0, nh])
        else:
            fr[24:26] = 0
            c = 0xffff - _csum(fr[14:34])
            fr[24:26] = [c >> 8, c & 0xff]
            nh, l4 = int(fr[23]), 34
            pseudo = bytes(fr[26:34]) + bytes([0, nh]) + (L - 34).to_bytes(2, "big")
        co = {TCP: 16, UDP: 6, ICMPV6: 2, ICMP: 2}[nh]
        fr[l4 + co:l4 + co + 2] = 0
        c = 0xffff - _csum((pseudo if nh != ICMP else b"") + bytes(fr[l4:L]))
        if nh == UDP and c == 0:
            c = 0xffff
        fr[l4 + co:l4 + co + 2] = [c >> 8, c & 0xff]
    sc.batches.append(synth.Packets(f, lens, None, None, None, np.zeros(n, np.uint8),
                                    rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)))
    return sc


def test_rewrites_keep_checksums_valid():
    sc = _scenario()
    pk = sc.batches[0]
    out, nd6, snap = OracleDP(sc).pipeline(pk, sc.now)
    reached = out["stage"] == 4
    assert ((out["flags"] & 0x40) != 0)[reached].sum() > 200          # translated
    assert ((out["flags"] & 0x80) != 0)[reached].sum() > 100          # port-mapped
    checked = 0
    for r in np.nonzero(reached)[0]:
        fr, L = snap[r], int(pk.lens[r])
        if fr[12] == 0x08:
            assert _csum(fr[14:34]) == 0xffff, r                       # IPv4 header checksum still valid
            nh, l4 = int(fr[23]), 34
            pseudo = bytes(fr[26:34]) + bytes([0, nh]) + (L - 34).to_bytes(2, "big")
            assert fr[22] == pk.frames[r, 22] - 1                      # TTL decremented
        else:
            nh, l4 = int(fr[20]), 54
            pseudo = bytes(fr[22:54]) + (L - 54).to_bytes(4, "big") + bytes([0, 0, 0, nh])
            assert fr[21] == pk.frames[r, 21] - 1
        assert bytes(fr[0:6]) == b"\xaa" * 6 and bytes(fr[6:12]) == b"\xbb" * 6
        if nh == ICMP:
            continue
        s = _csum(pseudo + bytes(fr[l4:L]))
        # the L3-fallback translation updates the L4 checksum from port 0 (key->dport was
        # zeroed, bpf/lib/lb.h:566-597 + l4_modify_port): the sum misses exactly the old port
        old_dport = int.from_bytes(bytes(pk.frames[r, l4 + 2:l4 + 4]), "big")
        fallback = bool(out["flags"][r] & 0x40) and out["dport"][r] != 0 and _lb_l3_fallback(sc, pk, r)
        if fallback:
            s2 = s + old_dport
            s2 = (s2 & 0xffff) + (s2 >> 16)
            assert s2 in (0xffff, 0), r
        else:
            assert s == 0xffff, (r, hex(s))
        checked += 1
    assert checked > 300


def _lb_l3_fallback(sc, pk, r):
    fr = pk.frames[r]
    v4, v6 = sc.meta["l3_only"]                                        # the L3-only services (port 0)
    if fr[12] == 0x08:
        return int.from_bytes(bytes(fr[30:34]), "big") == v4
    return bytes(fr[38:54]) == v6
