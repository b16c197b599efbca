"""Pins the CPU oracle: the reference's own known answers (test/bpf/unit-test.c)
plus hand-derived known answers read off the reference source (cited)."""
import ctypes as C
import struct

import numpy as np
import pytest

from cilium_amd import synth
from cilium_amd.synth import ip4, raw16, TCP, UDP, ICMP, F_SYN, F_ACK, F_FIN, F_RST
from oracle import oracle as O
from oracle.scenario import OracleDP


def htonl(x):
    return struct.unpack("<I", struct.pack(">I", x))[0]


# ---- test/bpf/unit-test.c:20-58 ----
@pytest.mark.parametrize("prefix,p", [(128, [0xffffffff] * 4), (127, [0xffffffff] * 3 + [0xfffffffe]),
                                      (95, [0xffffffff, 0xffffffff, 0xfffffffe, 0]), (1, [0x80000000, 0, 0, 0]),
                                      (-1, [0, 0, 0, 0])])
def test_ipv6_addr_clear_suffix_kat(prefix, p):
    a = (C.c_uint8 * 16)(*([0xff] * 16))
    O.lib.o_ipv6_addr_clear_suffix(a, prefix)
    words = struct.unpack(">4I", bytes(a))
    assert list(words) == p


# ---- test/bpf/unit-test.c:60-102 (LPM_LOOKUP_FN over explicit prefix lists) ----
def _lk(stored, prefixes, addr):
    arr = (C.c_int * len(prefixes))(*prefixes)
    return O.lib.o_lpm4_iter_lookup(htonl(stored), arr, len(prefixes), htonl(addr))


def test_lpm_lookup_kat():
    assert _lk(0xFFFFFFFF, [32], 0xFFFFFFFF)
    assert not _lk(0xFFFFFFFF, [32], 0xFFF00000)
    assert _lk(0xFFFFFFFE, [31], 0xFFFFFFFE)
    assert _lk(0xFFFFFFFE, [31], 0xFFFFFFFF)
    assert not _lk(0xFFFFFFFE, [31], 0xFFF00000)
    assert _lk(0xFFFFFC00, [22], 0xFFFFFC00)
    assert _lk(0xFFFFFC00, [22], 0xFFFFFFFF)
    assert not _lk(0xFFFFFC00, [22], 0xFFF00000)
    assert _lk(0xFFE00000, [11], 0xFFE00000)
    assert _lk(0xFFE00000, [11], 0xFFFFFFFF)
    assert _lk(0xFFE00000, [11], 0xFFF00000)
    assert _lk(0xF0000000, [11], 0xF0000000)
    assert _lk(0x00000000, [0], 0x00000000)
    assert _lk(0x00000000, [0], 0xFFFFFFFF)


# ---- hand-derived scenario KATs ----
E, R, VIP = ip4("10.1.0.5"), ip4("100.64.1.9"), ip4("10.96.0.10")
NOW = 7000


def _scn():
    sc = synth.Scenario("kat", now=NOW)
    sc.add_map(synth.MapSpec("ct4", synth.LRU_HASH, 14, 48, 1000, 0, np.zeros((0, 14), np.uint8),
                             np.zeros((0, 48), np.uint8)))
    keys = np.concatenate([synth.policy_keys([300], [0], [0]), synth.policy_keys([301], [80], [TCP]),
                           synth.policy_keys([302], [443], [TCP]), synth.policy_keys([0], [53], [UDP])])
    vals = np.concatenate([synth.policy_vals([0]), synth.policy_vals([0]), synth.policy_vals([15001]),
                           synth.policy_vals([0])])
    sc.add_map(synth.MapSpec("pol", synth.HASH, 8, 24, 16384, 0, keys, vals))
    ck, cv = synth.lpm4_keys([24], [ip4("100.64.1.0")]), np.ones((1, 1), np.uint8)
    sc.add_map(synth.MapSpec("cidr", synth.LPM, 8, 1, 100, 1, ck, cv))
    sc.add_map(synth.MapSpec("revnat", synth.HASH, 2, 6, 100, 0, np.zeros((0, 2), np.uint8), np.zeros((0, 6), np.uint8)))
    sc.lxc.append({"lxc_id": 7, "seclabel": 500, "policy": "pol", "ct4": "ct4", "ct6": None, "cidr4": "cidr",
                   "cidr6": None, "revnat4": "revnat", "revnat6": None, "flags": synth.LXC_PRODUCTION, "l4": []})
    sc.host_ifindex = 1
    return sc


def _pk(saddr, daddr, proto, sport, dport, flags, ident, icmp_type=8, lens=None, tc=0):
    f, l = synth.frames_v4(1, 64, [saddr], [daddr], [proto], [sport], [dport], [flags], [icmp_type], payload=10)
    if lens is not None:
        l = np.array([lens], np.uint32)
    return synth.Packets(f, l, np.array([ident], np.uint32), np.array([42], np.uint32), np.array([7], np.uint16),
                         np.array([tc], np.uint8))


def _ct(o):
    out = {}
    for k, v in o.dump("ct4").items():
        d, s, dp, sp, nh, fl = struct.unpack("<IIHHBB", k)
        e = struct.unpack("<QQQQIHHHHI", v)
        out[(d, s, dp, sp, nh, fl)] = dict(rx=e[0], rxb=e[1], life=e[4], flags=e[5], revnat=e[6], src=e[9])
    return out


def test_tcp_flow_lifecycle_kat():
    """conntrack.h:319-435 + 503-580, bpf_lxc.c:865-970 for an L3-allowed identity."""
    o = OracleDP(_scn())
    syn = _pk(R, E, TCP, 40000, 8080, F_SYN, 300)
    r = o.ingress(syn, NOW)[0]
    assert (r["action"], r["reason"], r["ct_ret"], r["flags"]) == (7, 0, 0, 2)     # redirect to ifindex 42
    ct = _ct(o)
    fwd = (htonl(R), htonl(E), raw16(8080), raw16(40000), TCP, 1)                  # reversed tuple, TUPLE_F_IN
    rel = (htonl(R), htonl(E), 0, 0, ICMP, 3)                                      # ICMP related, IN|RELATED
    assert set(ct) == {fwd, rel}
    assert ct[fwd]["life"] == NOW + 300 and ct[fwd]["flags"] == 0                  # SYN: CT_SYN_TIMEOUT
    assert ct[rel]["life"] == NOW + 300 and ct[rel]["flags"] == 16                 # seen_non_syn, same lifetime
    assert ct[fwd]["rx"] == 1 and ct[fwd]["rxb"] == syn.lens[0] and ct[fwd]["src"] == 300
    ack = _pk(R, E, TCP, 40000, 8080, F_ACK, 300)
    r = o.ingress(ack, NOW + 5)[0]
    assert (r["action"], r["ct_ret"]) == (7, 1)                                    # ESTABLISHED
    ct = _ct(o)
    assert ct[fwd]["life"] == NOW + 5 + 43200 and ct[fwd]["flags"] == 16 and ct[fwd]["rx"] == 2
    fin = _pk(R, E, TCP, 40000, 8080, F_FIN | F_ACK, 300)
    o.ingress(fin, NOW + 6)
    assert _ct(o)[fwd]["flags"] == 16 | 1                                          # rx_closing, still alive
    syn2 = _pk(R, E, TCP, 40000, 8080, F_SYN, 300)                                 # CREATE resets closing
    o.ingress(syn2, NOW + 7)
    c = _ct(o)[fwd]
    assert c["flags"] == 16 and c["life"] == NOW + 7 + 43200


def test_reply_direction_is_not_reply_at_ingress_kat():
    o = OracleDP(_scn())
    o.ingress(_pk(R, E, TCP, 40000, 8080, F_SYN, 300), NOW)
    r = o.ingress(_pk(E, R, TCP, 8080, 40000, F_ACK, 300), NOW)[0]
    assert r["ct_ret"] == 0                                                        # ingress of the reverse flow is NEW


def test_policy_kats():
    o = OracleDP(_scn())
    # L4 allow (301, 80/TCP) without proxy
    r = o.ingress(_pk(R, E, TCP, 1, 80, F_SYN, 301), NOW)[0]
    assert (r["action"], r["reason"], r["flags"] & 1) == (7, 0, 0)
    # L4 allow with proxy_port 15001 -> redirect to HOST_IFINDEX (1), proxy port reported raw be16
    r = o.ingress(_pk(R, E, TCP, 1, 443, F_SYN, 302), NOW)[0]
    assert (r["action"], r["flags"] & 1, r["proxy_port"], r["ifindex_lo"]) == (7, 1, raw16(15001), 1)
    # tc_index skip-proxy bit -> verdict forced to 0 (no proxy redirect)
    r = o.ingress(_pk(R, E, TCP, 2, 443, F_SYN, 302, tc=1), NOW)[0]
    assert (r["flags"] & 1, r["ifindex_lo"]) == (0, 42)
    # L4 wildcard {0, 53, UDP}
    r = o.ingress(_pk(R, E, UDP, 5, 53, 0, 999), NOW)[0]
    assert r["reason"] == 0
    # deny
    r = o.ingress(_pk(R, E, TCP, 1, 81, F_SYN, 301), NOW)[0]
    assert (r["action"], r["reason"]) == (2, 133)
    # reserved identity allowed by CIDR (100.64.1.0/24 covers R), denied outside
    r = o.ingress(_pk(R, E, TCP, 1, 81, F_SYN, 2), NOW)[0]
    assert r["reason"] == 0
    r = o.ingress(_pk(ip4("100.64.9.9"), E, TCP, 1, 81, F_SYN, 2), NOW)[0]
    assert r["reason"] == 133
    # user identity never uses CIDR
    r = o.ingress(_pk(R, E, TCP, 1, 81, F_SYN, 999), NOW)[0]
    assert r["reason"] == 133


def test_header_error_kats():
    o = OracleDP(_scn())
    assert o.ingress(_pk(R, E, TCP, 1, 80, F_SYN, 301, lens=33), NOW)[0]["reason"] == 134      # revalidate_data
    assert o.ingress(_pk(R, E, TCP, 1, 80, F_SYN, 301, lens=34 + 13), NOW)[0]["reason"] == 135  # tcp flags past len
    assert o.ingress(_pk(R, E, 47, 1, 80, 0, 301), NOW)[0]["reason"] == 137                     # unknown proto
    pk = _pk(R, E, TCP, 1, 80, F_SYN, 301)
    pk.lxc_id[:] = 8                                                                          # no program in slot
    assert o.ingress(pk, NOW)[0]["reason"] == 140


def test_lb_kats():
    """bpf_lb.c handle_ipv4 + lb.h lookup/select/xlate."""
    sc = synth.Scenario("lbkat")
    keys = np.concatenate([synth.lb4_keys([VIP], [80], [0]), synth.lb4_keys([VIP], [80], [1]),
                           synth.lb4_keys([VIP], [80], [2]), synth.lb4_keys([VIP], [80], [3]),
                           synth.lb4_keys([VIP], [0], [0]), synth.lb4_keys([VIP], [0], [1])])
    vals = np.concatenate([synth.lb4_vals([0], [0], [3], [0]), synth.lb4_vals([ip4("10.0.0.1")], [80], [0], [5]),
                           synth.lb4_vals([ip4("10.0.0.2")], [8080], [0], [5]),
                           synth.lb4_vals([ip4("10.0.0.3")], [80], [0], [5]), synth.lb4_vals([0], [0], [2], [0]),
                           synth.lb4_vals([ip4("10.0.0.9")], [7000], [0], [6])])
    sc.add_map(synth.MapSpec("svc", synth.HASH, 8, 12, 100, 0, keys, vals))
    sc.lb = {"lb4": "svc", "lb6": None, "flags": synth.LB_L3 | synth.LB_L4 | synth.LB_REDIRECT, "redirect_ifindex": 1}
    o = OracleDP(sc)

    def run(dport, h, proto=TCP, lens=None):
        f, l = synth.frames_v4(1, 64, [E], [VIP], [proto], [1234], [dport], [F_ACK], payload=10)
        if lens is not None:
            l = np.array([lens], np.uint32)
        return o.lb(synth.Packets(f, l, flow_hash=np.array([h], np.uint32)))[0][0]

    r = run(80, 4)                              # slave = 4 % 3 + 1 = 2 -> 10.0.0.2:8080, port rewritten
    assert (r["action"], r["slave"], r["new_daddr4"], r["new_dport"]) == (7, 2, htonl(ip4("10.0.0.2")), raw16(8080))
    r = run(80, 5)                              # slave 3, same port -> no rewrite
    assert (r["slave"], r["new_dport"]) == (3, 0)
    r = run(81, 1)                              # L4 miss -> key.dport = 0 -> L3 service, count 2, slave 2 missing
    assert (r["action"], r["reason"]) == (2, 158)
    r = run(81, 0)                              # L3 slave 1 -> port rewrite with old_port 0 (lb.h:648-655 quirk)
    assert (r["action"], r["slave"], r["new_dport"]) == (7, 1, raw16(7000))
    r = run(80, 4, lens=14 + 20 + 3)            # dport load past len -> -EFAULT
    assert (r["action"], r["reason"]) == (2, 14)
    r = run(80, 4, lens=14 + 20 + 10)           # TCP csum field (l4+16) past len -> DROP_CSUM_L4
    assert (r["action"], r["reason"]) == (2, 154)


def test_xdp_kats():
    sc = synth.Scenario("xdpkat")
    sc.add_map(synth.MapSpec("dyn", synth.LPM, 8, 1, 100, 1, synth.lpm4_keys([24, 8], [ip4("1.2.3.0"), ip4("44.0.0.0")]),
                             np.ones((2, 1), np.uint8)))
    sc.add_map(synth.MapSpec("fix", synth.HASH, 8, 1, 100, 1, synth.lpm4_keys([32], [ip4("5.6.7.8")]),
                             np.ones((1, 1), np.uint8)))
    sc.add_map(synth.MapSpec("lxc", synth.HASH, 20, 112, 100, 0, synth.endpoint_keys4([E]),
                             synth.endpoint_infos([1], [2], [3], [0])))
    sc.xdp = {"cidr4_hmap": "fix", "cidr4_lmap": "dyn", "lxc_map": "lxc"}
    o = OracleDP(sc)

    def run(s, d, lens=None, et=None):
        f, l = synth.frames_v4(1, 64, [s], [d], [TCP], [1], [2], [F_ACK], payload=0)
        if lens is not None:
            l = np.array([lens], np.uint32)
        if et is not None:
            f[0, 12], f[0, 13] = et >> 8, et & 0xff
        return int(o.xdp(synth.Packets(f, l))[0])

    assert run(ip4("9.9.9.9"), E) == 2                       # endpoint -> PASS
    assert run(ip4("9.9.9.9"), ip4("9.9.9.10")) == 1         # not an endpoint -> DROP
    assert run(ip4("1.2.3.77"), E) == 1                      # LPM /24 hit -> DROP
    assert run(ip4("44.200.1.1"), E) == 1                    # LPM /8 hit -> DROP
    assert run(ip4("5.6.7.8"), E) == 1                       # /32 hash hit -> DROP
    assert run(ip4("9.9.9.9"), E, lens=33) == 1              # xdp_no_room
    assert run(ip4("9.9.9.9"), E, lens=13) == 1              # shorter than an Ethernet header
    assert run(ip4("9.9.9.9"), E, et=0x0806) == 2            # ARP -> PASS
