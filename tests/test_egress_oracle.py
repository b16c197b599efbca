"""Hand-derived known answers for the from-container restatement
(bpf/bpf_lxc.c:427-738 handle_ingress -> handle_ipv4_from_lxc), read off the
reference text (cited per case), plus the egress fuzz scenario's invariants."""
import struct

import numpy as np

from cilium_amd import synth
from cilium_amd.synth import ip4, TCP, F_SYN, F_ACK
from oracle.scenario import OracleDP

S, PEER, VIP, VIP2, LOOP = ip4("10.1.0.5"), ip4("10.1.0.6"), ip4("10.96.0.10"), ip4("10.96.0.11"), ip4("10.255.255.245")
WORLD, TUN = ip4("100.64.1.9"), ip4("10.128.3.4")
NOW = 9000
LXC_MAC = bytes([0xaa, 0xbb, 0xcc, 0, 0, 5])
NODE_MAC = bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])
HOST_MAC = bytes([0xce, 0x72, 0xa7, 0x03, 0x88, 0x56])


def raw_be(a):
    return int(synth.be32_bytes([a]).view("<u4")[0, 0])


def _scn(policy_egress=False):
    sc = synth.Scenario("egkat", now=NOW, host_ifindex=3)
    M = synth.MapSpec
    sc.add_map(M("ct4", synth.LRU_HASH, 14, 48, 1000, 0))
    sc.add_map(M("ct6", synth.LRU_HASH, 40, 48, 1000, 0))
    for e in (0, 1):
        sc.add_map(M(f"pol{e}", synth.HASH, 8, 24, 1024, 0, synth.policy_keys([256, 300, 301], [0] * 3, [0] * 3),
                     synth.policy_vals([0] * 3)))
    ek = synth.endpoint_keys4(np.array([S, PEER], np.uint32))
    ev = synth.endpoint_infos([20, 21], [300, 301], [100, 101], [0, 0])
    ev[0, 16:22] = list(LXC_MAC)
    ev[:, 24:30] = list(NODE_MAC)
    sc.add_map(M("cilium_lxc", synth.HASH, 20, 112, 1024, 0, ek, ev))
    k = np.concatenate([synth.lb4_keys([VIP], [80], [0]), synth.lb4_keys([VIP], [80], [1]),
                        synth.lb4_keys([VIP2], [80], [0]), synth.lb4_keys([VIP2], [80], [1])])
    v = np.concatenate([synth.lb4_vals([0], [0], [1], [0]), synth.lb4_vals([S], [8080], [0], [7]),
                        synth.lb4_vals([0], [0], [1], [0]), synth.lb4_vals([PEER], [80], [0], [8])])
    sc.add_map(M("lb4", synth.HASH, 8, 12, 1024, 0, k, v))
    rk, rv = synth.revnat4_entries([7, 8], np.array([VIP, VIP2], np.uint32), [80, 80])
    sc.add_map(M("revnat4", synth.HASH, 2, 6, 1024, 0, rk, rv))
    sc.add_map(M("tunnel", synth.HASH, 20, 20, 64, 0, synth.endpoint_keys4(np.array([ip4("10.128.0.0")], np.uint32)),
                 synth.endpoint_keys4(np.array([ip4("192.168.7.2")], np.uint32))))
    sc.add_map(M("cilium_proxy4", synth.HASH, 10, 16, 1024, 0))
    for e, ip in ((0, S), (1, PEER)):
        sc.lxc.append({"lxc_id": 100 + e, "seclabel": 300 + e, "policy": f"pol{e}", "ct4": "ct4", "ct6": "ct6",
                       "revnat4": "revnat4", "flags": synth.LXC_PRODUCTION | (synth.LXC_POLICY_EGRESS if policy_egress else 0),
                       "lxc_mac": LXC_MAC if e == 0 else bytes(6), "node_mac": NODE_MAC, "lxc_ipv4": raw_be(ip),
                       "lb4": "lb4"})
    sc.node = {"proxy4": "cilium_proxy4", "ipv4_gateway": raw_be(ip4("10.255.0.1")), "host_mac": HOST_MAC,
               "node_mac": NODE_MAC, "lxc_map": "cilium_lxc", "ipv4_cluster_range": raw_be(ip4("10.0.0.0")),
               "ipv4_cluster_mask": raw_be(0xFF000000), "ipv4_loopback": raw_be(LOOP), "ipv4_mask": raw_be(0xFFFF0000),
               "encap_ifindex": 5, "tunnel_map": "tunnel"}
    return sc


def _pk(daddr, dport, flags=F_SYN, saddr=S, smac=LXC_MAC, ttl=64, proto=TCP, sport=40000):
    f, lens = synth.frames_v4(1, 128, [saddr], [daddr], [proto], [sport], [dport], [flags])
    f[0, 0:6] = list(NODE_MAC)
    f[0, 6:12] = list(smac)
    f[0, 22] = ttl
    return synth.Packets(f, lens, None, None, np.array([100], np.uint16), None, np.array([0], np.uint32))


def _ct(ref):
    out = {}
    for k, v in ref.dump("ct4").items():
        d, s, dp, sp, nh, fl = struct.unpack(">IIHHBB", k)
        rxp, rxb, txp, txb, life, ef, rn = struct.unpack("<QQQQIHH", v[:40])
        out[(d, s, dp, sp, nh, fl)] = dict(tx=(txp, txb), rx=(rxp, rxb), life=life, flags=ef,
                                           src_sec=struct.unpack("<I", v[44:48])[0])
    return out


def test_syn_to_world_passes_to_stack_and_creates_ct():
    """bpf_lxc.c:499-545 (ct_lookup4 CT_EGRESS -> CT_NEW -> ct_create4 with tx
    counters, conntrack.h:503-580), :640-657 pass_to_stack (ipv4_l3: TTL - 1,
    dmac = NODE_MAC)."""
    ref = OracleDP(_scn())
    pk = _pk(WORLD, 443)
    o, snap = ref.egress(pk, NOW)
    o = o[0]
    assert (o["stage"], o["action"], o["eg_ct_ret"]) == (5, 0, 0)
    assert o["eg_flags"] == 0x0001 | 0x0100                     # CREATED | TO_STACK
    ct = _ct(ref)
    n = int(pk.lens[0])
    # forward tuple after ipv4_ct_tuple_reverse: {daddr = sender, saddr = peer, dport, sport, OUT}
    e = ct[(S, WORLD, 443, 40000, TCP, 0)]
    assert e["tx"] == (1, n) and e["rx"] == (0, 0) and e["life"] == NOW + 300 and e["src_sec"] == 300
    rel = ct[(S, WORLD, 0, 0, 1, 2)]                             # ICMP related entry, seen_non_syn
    assert rel["flags"] & 16 and rel["life"] == NOW + 300
    assert len(ct) == 2
    assert snap[0, 22] == 63 and bytes(snap[0, 0:6]) == NODE_MAC
    o2, _ = ref.egress(_pk(WORLD, 443, F_ACK), NOW + 5)
    assert o2[0]["eg_ct_ret"] == 1                               # CT_ESTABLISHED
    e = _ct(ref)[(S, WORLD, 443, 40000, TCP, 0)]
    assert e["tx"][0] == 2 and e["life"] == NOW + 5 + 43200


def test_source_checks():
    """is_valid_lxc_src_mac / is_valid_gw_dst_mac / is_valid_lxc_src_ipv4 (lib/lxc.h:32-88)."""
    ref = OracleDP(_scn())
    assert ref.egress(_pk(WORLD, 80, smac=bytes(6)), NOW)[0][0]["reason"] == 130
    p = _pk(WORLD, 80)
    p.frames[0, 0] ^= 1
    assert ref.egress(p, NOW)[0][0]["reason"] == 131
    assert ref.egress(_pk(WORLD, 80, saddr=PEER), NOW)[0][0]["reason"] == 132


def test_service_loopback_to_sender():
    """lb4_local's loopback branch (lib/lb.h:662-699): saddr -> IPV4_LOOPBACK,
    daddr -> the backend (the sender), tuple daddr stays the VIP; ct_create4
    writes the loopback entry {IPV4_LOOPBACK, sender, IN} (conntrack.h:533-561);
    the frame is delivered back to the sender (l3.h:136-168)."""
    ref = OracleDP(_scn())
    o, snap = ref.egress(_pk(VIP, 80), NOW)
    o = o[0]
    assert o["eg_flags"] & 0x000C == 0x000C and o["slave"] == 1   # LB | LOOPBACK
    assert struct.unpack(">II", bytes(snap[0, 26:34])) == (LOOP, S)
    assert struct.unpack(">H", bytes(snap[0, 36:38]))[0] == 8080
    ct = _ct(ref)
    assert (S, VIP, 8080, 40000, TCP, 0) in ct
    lo = ct[(LOOP, S, 8080, 40000, TCP, 1)]
    assert lo["flags"] & 8                                       # lb_loopback
    assert o["stage"] == 4 and o["lxc_id"] == 100                 # handle_policy of the sender itself
    # whose ct_lookup4(CT_INGRESS) finds the loopback entry as the forward tuple
    assert (o["action"], o["ct_ret"]) == (7, 1) and lo["rx"] == (1, int(54))


def test_service_to_peer_and_service_entry():
    """lb4_local without loopback: tuple daddr = backend; the service entry of
    ct_create4 gets daddr = ct_state->addr = the backend, i.e. {backend, backend}."""
    ref = OracleDP(_scn())
    o, snap = ref.egress(_pk(VIP2, 80), NOW)
    o = o[0]
    assert o["stage"] == 4 and o["lxc_id"] == 101 and o["rev_nat"] == synth.raw16([8])[0]
    ct = _ct(ref)
    assert (S, PEER, 80, 40000, TCP, 0) in ct and (PEER, PEER, 80, 40000, TCP, 0) in ct


def test_tunnel_encap():
    """encap_and_redirect (lib/encap.h): daddr & IPV4_MASK in cilium_tunnel_map ->
    redirect(ENCAP_IFINDEX) with the tunnel key's remote_ipv4 = bpf_htonl(tunnel->ip4)."""
    ref = OracleDP(_scn())
    o = ref.egress(_pk(TUN, 80), NOW)[0][0]
    assert (o["action"], o["ifindex_lo"]) == (7, 5) and o["eg_flags"] & 0x0040
    assert o["tunnel_ip"] == ip4("192.168.7.2")


def test_policy_egress_cidr_default_deny():
    """policy_can_egress4 with POLICY_EGRESS (policy.h:241-264): WORLD is reserved,
    no policy entry, no CIDR4_EGRESS_MAP -> DROP_POLICY_CIDR (maps.h:240-243)."""
    ref = OracleDP(_scn(policy_egress=True))
    o = ref.egress(_pk(WORLD, 443), NOW)[0][0]
    assert (o["action"], o["reason"]) == (2, 162)
    assert _ct(ref) == {}


def test_fuzz_invariants():
    sc = synth.egress_fuzz(seed=5, n_packets=5000, n_batches=2)
    ref = OracleDP(sc)
    for bi, pk in enumerate(sc.batches):
        o, _ = ref.egress(pk, sc.now + bi)
        st = o["stage"]
        assert set(np.unique(st)) == {0, 4, 5}
        assert np.all(o["action"][st == 0] == 0)
        shot = o["action"] == 2
        assert np.all(o["reason"][shot] > 0) and np.all(o["reason"][~shot] == 0)
        assert np.all((o["eg_flags"][st == 4] & 0x0200) != 0)


def test_ipv6_pass_to_stack_flowlabel_and_responders():
    """ipv6_l3_from_lxc's pass_to_stack (bpf_lxc.c:370-385): hop limit - 1, dmac =
    NODE_MAC, ipv6_store_flowlabel(SECLABEL_NB) keeping the traffic class
    (bpf/lib/ipv6.h:245-260); icmp6_handle's NS goes to the responder (stage NONE)."""
    sc = _scn()
    s6 = bytes([0xf0, 0x0d] + [0] * 13 + [5])
    d6 = bytes([0x20, 0x01, 0x0d, 0xb8] + [0] * 11 + [9])
    sc.lxc[0]["lxc_ip6"] = s6
    ref = OracleDP(sc)
    f, lens = synth.frames_v6(2, 128, np.frombuffer(s6, np.uint8), np.frombuffer(d6, np.uint8),
                              np.array([TCP, 58], np.uint8), 40000, 443, F_SYN, 135)
    f[:, 0:6] = list(NODE_MAC)
    f[:, 6:12] = list(LXC_MAC)
    f[:, 15] = 0x3c                                     # traffic class bits in the first word
    pk = synth.Packets(f, lens, None, None, np.array([100, 100], np.uint16), None, np.zeros(2, np.uint32))
    o, snap = ref.egress(pk, NOW)
    assert (o[0]["stage"], o[0]["action"]) == (5, 0) and o[0]["eg_flags"] == 0x1000 | 0x0100 | 0x0001
    word = struct.unpack(">I", bytes(snap[0, 14:18]))[0]
    assert word == 0x60000000 | (0x0FF00000 & struct.unpack(">I", bytes(f[0, 14:18]))[0]) | 300
    assert snap[0, 21] == 63 and bytes(snap[0, 0:6]) == NODE_MAC
    assert o[1]["stage"] == 0 and o[1]["eg_flags"] == 0x1000 | 0x4000
