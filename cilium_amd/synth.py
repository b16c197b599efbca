"""Seeded synthetic workloads (BASELINE.json configs 1-5 + a parity fuzz set).

Every scenario is plain data: map contents as key/value byte arrays in the
reference layouts (bpf/lib/common.h), program configurations, and a batch of
raw Ethernet frames plus the skb metadata the calling programs provide.  The
same Scenario is installed into libgpuflow (cilium_amd.datapath) and into the
CPU oracle (tests / bench cpu_baseline), so both see identical inputs.

Addresses are host-order integers here; frames and keys carry network order.
"""
from dataclasses import dataclass, field
import struct

import numpy as np

# map types / flags (pkg/bpf/bpf.go)
HASH, LRU_HASH, LPM = 1, 9, 11
NO_PREALLOC = 1
# program flags (include/gpuflow.h)
LB_L3, LB_L4, LB_REDIRECT, LB_NO_IPV4, LB_NO_IPV6 = 1, 2, 4, 8, 16
LXC_DROP_ALL, LXC_POLICY_INGRESS, LXC_HAVE_L4_POLICY, LXC_CT_ACCOUNTING, LXC_LXC_IPV4 = 1, 2, 4, 8, 16
LXC_PRODUCTION = LXC_POLICY_INGRESS | LXC_HAVE_L4_POLICY | LXC_CT_ACCOUNTING | LXC_LXC_IPV4
TCP, UDP, ICMP, ICMPV6 = 6, 17, 1, 58
F_FIN, F_SYN, F_RST, F_PSH, F_ACK = 0x01, 0x02, 0x04, 0x08, 0x10


@dataclass
class MapSpec:
    name: str
    type: int
    ksz: int
    vsz: int
    max_entries: int
    flags: int = 0
    keys: np.ndarray = None      # uint8 [n, ksz]
    vals: np.ndarray = None      # uint8 [n, vsz]

    def n(self):
        return 0 if self.keys is None else self.keys.shape[0]


@dataclass
class Packets:
    frames: np.ndarray           # uint8 [n, stride]
    lens: np.ndarray             # uint32 [n]
    src_identity: np.ndarray = None
    ifindex: np.ndarray = None
    lxc_id: np.ndarray = None
    tc_index: np.ndarray = None
    flow_hash: np.ndarray = None

    @property
    def n(self):
        return self.frames.shape[0]

    def slice(self, a, b):
        f = lambda x: None if x is None else x[a:b]
        return Packets(self.frames[a:b], self.lens[a:b], f(self.src_identity), f(self.ifindex), f(self.lxc_id),
                       f(self.tc_index), f(self.flow_hash))


@dataclass
class Scenario:
    name: str
    maps: dict = field(default_factory=dict)
    xdp: dict = None             # role -> map name
    lb: dict = None              # {'lb4','lb6','flags','redirect_ifindex'}
    lxc: list = field(default_factory=list)   # endpoint program configs
    netdev: dict = None          # bpf_netdev config of the full pipeline (gf_netdev_cfg)
    node: dict = None            # node_config.h values beyond HOST_IFINDEX (gf_node_cfg): proxy maps, ...
    host_ifindex: int = 1
    batches: list = field(default_factory=list)   # list of Packets, processed in order
    now: int = 1000
    meta: dict = field(default_factory=dict)

    def add_map(self, spec):
        self.maps[spec.name] = spec
        return spec


# ------------------------------------------------------------------ helpers
def be32_bytes(a):
    """host-order u32 array -> uint8 [n,4] network order."""
    a = np.asarray(a, dtype=np.uint32)
    return a.astype(">u4").view(np.uint8).reshape(-1, 4)


def be16_bytes(a):
    a = np.asarray(a, dtype=np.uint16)
    return a.astype(">u2").view(np.uint8).reshape(-1, 2)


def raw16(a):
    """host-order port -> the u16 a BPF program holds after loading the be16 (LE view)."""
    a = np.asarray(a, dtype=np.uint32)
    return (((a & 0xff) << 8) | (a >> 8)).astype(np.uint16)


def le_bytes(a, dt):
    return np.ascontiguousarray(np.asarray(a, dtype=dt)).view(np.uint8).reshape(len(a), -1)


def pack_rows(*cols):
    """Concatenate uint8 [n, k] column blocks into [n, sum k]."""
    return np.ascontiguousarray(np.concatenate(cols, axis=1))


def mix32(x):
    x = np.asarray(x, dtype=np.uint64)
    x = (x ^ (x >> np.uint64(33))) * np.uint64(0xff51afd7ed558ccd)
    x = (x ^ (x >> np.uint64(33))) * np.uint64(0xc4ceb9fe1a85ec53)
    x ^= x >> np.uint64(33)
    return (x & np.uint64(0xffffffff)).astype(np.uint32)


def ip4(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


# ------------------------------------------------------------------ frames
def frames_v4(n, stride, saddr, daddr, proto, sport=0, dport=0, tcp_flags=0, icmp_type=0, icmp_code=0,
              ihl=5, lens=None, payload=0):
    """Vectorised IPv4/Ethernet frames (headers inside the snap)."""
    f = np.zeros((n, stride), np.uint8)
    bc = lambda x, dt: np.broadcast_to(np.asarray(x, dtype=dt), (n,)).copy()
    saddr, daddr = bc(saddr, np.uint32), bc(daddr, np.uint32)
    proto, ihl = bc(proto, np.uint8), bc(ihl, np.uint32)
    sport, dport = bc(sport, np.uint32), bc(dport, np.uint32)
    tcp_flags, icmp_type, icmp_code = bc(tcp_flags, np.uint8), bc(icmp_type, np.uint8), bc(icmp_code, np.uint8)
    f[:, 0:6] = 0x02
    f[:, 6:12] = 0x04
    f[:, 12], f[:, 13] = 0x08, 0x00
    f[:, 14] = (0x40 | (ihl & 0xf)).astype(np.uint8)
    f[:, 22] = 64
    f[:, 23] = proto
    f[:, 26:30] = be32_bytes(saddr)
    f[:, 30:34] = be32_bytes(daddr)
    l4 = (14 + (ihl & 0xf) * 4).astype(np.int64)
    rows = np.arange(n)

    def put(off, val):
        ok = off < stride
        f[rows[ok], off[ok]] = np.asarray(val)[ok]

    is_tu = (proto == TCP) | (proto == UDP)
    put(np.where(is_tu, l4, stride), (sport >> 8).astype(np.uint8))
    put(np.where(is_tu, l4 + 1, stride), (sport & 0xff).astype(np.uint8))
    put(np.where(is_tu, l4 + 2, stride), (dport >> 8).astype(np.uint8))
    put(np.where(is_tu, l4 + 3, stride), (dport & 0xff).astype(np.uint8))
    is_tcp = proto == TCP
    put(np.where(is_tcp, l4 + 12, stride), np.full(n, 0x50, np.uint8))
    put(np.where(is_tcp, l4 + 13, stride), tcp_flags)
    is_icmp = (proto == ICMP) | (proto == ICMPV6)
    put(np.where(is_icmp, l4, stride), icmp_type)
    put(np.where(is_icmp, l4 + 1, stride), icmp_code)
    l4h = np.where(is_tcp, 20, np.where(proto == UDP, 8, np.where(is_icmp, 8, 0)))
    if lens is None:
        lens = (l4 + l4h + payload).astype(np.uint32)
    lens = np.asarray(lens, np.uint32)
    tot = np.minimum(lens - 14, 0xffff).astype(np.uint16)
    f[:, 16:18] = be16_bytes(tot)
    return f, lens


def frames_v6(n, stride, saddr6, daddr6, nexthdr, sport=0, dport=0, tcp_flags=0, icmp_type=0,
              ext=None, lens=None, payload=0):
    """Vectorised IPv6 frames.  ext: list of (types[n], hdrlen[n]) extension headers
    chained after the fixed header (type 255 = stop)."""
    f = np.zeros((n, stride), np.uint8)
    bc = lambda x, dt: np.broadcast_to(np.asarray(x, dtype=dt), (n,)).copy()
    nexthdr = bc(nexthdr, np.uint8)
    sport, dport = bc(sport, np.uint32), bc(dport, np.uint32)
    tcp_flags, icmp_type = bc(tcp_flags, np.uint8), bc(icmp_type, np.uint8)
    f[:, 12], f[:, 13] = 0x86, 0xDD
    f[:, 14] = 0x60
    f[:, 21] = 64
    f[:, 22:38] = saddr6
    f[:, 38:54] = daddr6
    rows = np.arange(n)

    def put(off, val):
        ok = (off >= 0) & (off < stride)
        f[rows[ok], off[ok]] = np.asarray(val)[ok]

    off = np.full(n, 54, np.int64)
    cur_field = np.full(n, 20, np.int64)      # where the "next header" byte of the current header lives
    final_nh = nexthdr.copy()
    active = np.ones(n, bool)
    first = True
    for (types, hlen) in (ext or []):
        types = bc(types, np.uint8)
        hlen = bc(hlen, np.uint8)
        act = active & (types != 255)
        # chain: previous header's nexthdr field points to this ext type
        if first:
            f[rows[act], 20] = types[act]
            first = False
        else:
            put(np.where(act, cur_field, -1), types)
        cur_field = np.where(act, off, cur_field)       # this header's nexthdr byte
        put(np.where(act, off + 1, -1), hlen)
        # real extension-header length as the kernel defines it
        ln = np.where(types == 51, (hlen.astype(np.int64) + 2) << 2, (hlen.astype(np.int64) + 1) << 3)
        off = np.where(act, off + ln, off)
        active = act
    if ext:
        # last header in the chain names the upper-layer protocol
        has = cur_field != 20
        put(np.where(has, cur_field, -1), final_nh)
        f[rows[~has], 20] = final_nh[~has]
    else:
        f[:, 20] = nexthdr
    l4 = off
    is_tu = (nexthdr == TCP) | (nexthdr == UDP)
    put(np.where(is_tu, l4, -1), (sport >> 8).astype(np.uint8))
    put(np.where(is_tu, l4 + 1, -1), (sport & 0xff).astype(np.uint8))
    put(np.where(is_tu, l4 + 2, -1), (dport >> 8).astype(np.uint8))
    put(np.where(is_tu, l4 + 3, -1), (dport & 0xff).astype(np.uint8))
    is_tcp = nexthdr == TCP
    put(np.where(is_tcp, l4 + 12, -1), np.full(n, 0x50, np.uint8))
    put(np.where(is_tcp, l4 + 13, -1), tcp_flags)
    is_icmp = (nexthdr == ICMPV6) | (nexthdr == ICMP)
    put(np.where(is_icmp, l4, -1), icmp_type)
    l4h = np.where(is_tcp, 20, np.where(nexthdr == UDP, 8, np.where(is_icmp, 8, 0)))
    if lens is None:
        lens = (l4 + l4h + payload).astype(np.uint32)
    lens = np.asarray(lens, np.uint32)
    f[:, 18:20] = be16_bytes(np.clip(lens.astype(np.int64) - 54, 0, 0xffff))
    return f, lens


def flow_hash(saddr, daddr, sport, dport, proto, seed=0x5eed):
    """Documented stand-in for the kernel's skb hash (get_hash_recalc has a
    per-boot secret seed, lb.h:109-121): a 5-tuple mix.  An INPUT column."""
    x = (np.asarray(saddr, np.uint64) << np.uint64(32)) ^ np.asarray(daddr, np.uint64)
    y = (np.asarray(sport, np.uint64) << np.uint64(24)) ^ (np.asarray(dport, np.uint64) << np.uint64(8)) ^ \
        np.asarray(proto, np.uint64)
    return mix32(mix32(x) .astype(np.uint64) * np.uint64(0x9E3779B1) ^ y ^ np.uint64(seed))


# ------------------------------------------------------------------ key/value builders
def lpm4_keys(prefixlen, net):
    return pack_rows(le_bytes(prefixlen, "<u4"), be32_bytes(net))


def lpm6_keys(prefixlen, net16):
    return pack_rows(le_bytes(prefixlen, "<u4"), np.asarray(net16, np.uint8).reshape(-1, 16))


def endpoint_keys4(ip):
    n = len(ip)
    return pack_rows(be32_bytes(ip), np.zeros((n, 12), np.uint8), np.ones((n, 1), np.uint8),
                     np.zeros((n, 3), np.uint8))


def endpoint_keys6(ip16):
    n = len(ip16)
    return pack_rows(np.asarray(ip16, np.uint8), np.full((n, 1), 2, np.uint8), np.zeros((n, 3), np.uint8))


def endpoint_infos(ifindex, sec_label, lxc_id, flags):
    n = len(ifindex)
    v = np.zeros((n, 112), np.uint8)
    v[:, 0:4] = le_bytes(ifindex, "<u4")
    v[:, 4:6] = le_bytes(sec_label, "<u2")
    v[:, 6:8] = le_bytes(lxc_id, "<u2")
    v[:, 8:12] = le_bytes(flags, "<u4")
    return v


def policy_keys(identity, dport_host, proto, egress=0):
    n = len(identity)
    return pack_rows(le_bytes(identity, "<u4"), le_bytes(raw16(dport_host), "<u2"),
                     np.asarray(proto, np.uint8).reshape(n, 1),
                     np.broadcast_to(np.asarray(egress, np.uint8), (n,)).reshape(n, 1))


def policy_vals(proxy_port_host):
    n = len(proxy_port_host)
    v = np.zeros((n, 24), np.uint8)
    pp = np.asarray(proxy_port_host, np.uint32)
    v[:, 0:2] = le_bytes(np.where(pp > 0, raw16(pp), 0), "<u2")
    return v


def ct4_keys(daddr, saddr, dport_raw, sport_raw, nexthdr, flags):
    n = len(daddr)
    return pack_rows(be32_bytes(daddr), be32_bytes(saddr), le_bytes(dport_raw, "<u2"), le_bytes(sport_raw, "<u2"),
                     np.asarray(nexthdr, np.uint8).reshape(n, 1), np.asarray(flags, np.uint8).reshape(n, 1))


def ct_vals(n, lifetime, flags=0, revnat=0, src_sec=0, rx=(0, 0), tx=(0, 0)):
    v = np.zeros((n, 48), np.uint8)
    v[:, 0:8] = le_bytes(np.broadcast_to(np.uint64(rx[0]), (n,)), "<u8")
    v[:, 8:16] = le_bytes(np.broadcast_to(np.uint64(rx[1]), (n,)), "<u8")
    v[:, 16:24] = le_bytes(np.broadcast_to(np.uint64(tx[0]), (n,)), "<u8")
    v[:, 24:32] = le_bytes(np.broadcast_to(np.uint64(tx[1]), (n,)), "<u8")
    v[:, 32:36] = le_bytes(np.broadcast_to(np.asarray(lifetime, np.uint32), (n,)), "<u4")
    v[:, 36:38] = le_bytes(np.broadcast_to(np.asarray(flags, np.uint16), (n,)), "<u2")
    v[:, 38:40] = le_bytes(np.broadcast_to(np.asarray(revnat, np.uint16), (n,)), "<u2")
    v[:, 44:48] = le_bytes(np.broadcast_to(np.asarray(src_sec, np.uint32), (n,)), "<u4")
    return v


def lb4_keys(addr, port_host, slave):
    return pack_rows(be32_bytes(addr), le_bytes(raw16(port_host), "<u2"), le_bytes(slave, "<u2"))


def lb4_vals(target, port_host, count, revnat_host, weight=0):
    n = len(target)
    w = np.broadcast_to(np.asarray(weight, np.uint32), (n,))
    return pack_rows(be32_bytes(target), le_bytes(raw16(port_host), "<u2"), le_bytes(count, "<u2"),
                     le_bytes(raw16(revnat_host), "<u2"), le_bytes(raw16(w), "<u2"))


def lb6_keys(addr16, port_host, slave):
    return pack_rows(np.asarray(addr16, np.uint8), le_bytes(raw16(port_host), "<u2"), le_bytes(slave, "<u2"))


def lb6_vals(target16, port_host, count, revnat_host, weight=0):
    n = len(target16)
    w = np.broadcast_to(np.asarray(weight, np.uint32), (n,))
    return pack_rows(np.asarray(target16, np.uint8), le_bytes(raw16(port_host), "<u2"), le_bytes(count, "<u2"),
                     le_bytes(raw16(revnat_host), "<u2"), le_bytes(raw16(w), "<u2"))


def revnat4_entries(ids_host, addr, port_host):
    k = le_bytes(raw16(ids_host), "<u2")
    v = pack_rows(be32_bytes(addr), le_bytes(raw16(port_host), "<u2"))
    return k, v


def revnat6_entries(ids_host, addr16, port_host):
    k = le_bytes(raw16(ids_host), "<u2")
    v = pack_rows(np.asarray(addr16, np.uint8), le_bytes(raw16(port_host), "<u2"))
    return k, v


def dedup(keys, vals):
    """Keep the LAST occurrence of each key (BPF_ANY update order)."""
    kv = np.ascontiguousarray(keys).view(np.dtype((np.void, keys.shape[1]))).ravel()
    _, idx = np.unique(kv[::-1], return_index=True)
    idx = np.sort(len(kv) - 1 - idx)
    return keys[idx], vals[idx]


def lpm_dedup(keys, vals, bits):
    """Normalise LPM keys (mask bits past prefixlen) and dedup (trie semantics)."""
    keys = keys.copy()
    plen = keys[:, 0:4].copy().view("<u4").ravel()
    nbytes = bits // 8
    for b in range(nbytes):
        keep = np.clip(plen.astype(np.int64) - 8 * b, 0, 8)
        mask = (0xff << (8 - keep)) & 0xff
        keys[:, 4 + b] &= mask.astype(np.uint8)
    return dedup(keys, vals)


def rand_v6(rng, n, prefix=(0x20, 0x01, 0x0d, 0xb8)):
    a = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    a[:, :len(prefix)] = prefix
    return a


# ------------------------------------------------------------------ config 1: XDP prefilter
def config1(n_packets=1_000_000, n_lpm=10_000, n_fix=2_000, n_ep=1_024, seed=0xC1D40001, stride=64):
    """BASELINE config 1 / SURVEY §8(d): bpf_xdp.c CIDR prefilter."""
    rng = np.random.default_rng(seed)
    sc = Scenario("config1_xdp")
    # v4_dyn: 55% /24, 25% /16-/23, 15% /25-/31, 5% /8-/15, with nesting
    u = rng.random(n_lpm)
    plen = np.where(u < 0.55, 24, np.where(u < 0.80, rng.integers(16, 24, n_lpm),
                                           np.where(u < 0.95, rng.integers(25, 32, n_lpm), rng.integers(8, 16, n_lpm))))
    net = rng.integers(0, 1 << 32, n_lpm, dtype=np.uint64).astype(np.uint32)
    # 20% nested: take the network of an earlier prefix and extend it
    nest = rng.random(n_lpm) < 0.20
    parent = rng.integers(0, n_lpm, n_lpm)
    net = np.where(nest, (net[parent] & ~((1 << (32 - np.minimum(plen[parent], 31))) - 1).astype(np.uint32)) |
                   (net & ((1 << (32 - np.minimum(plen[parent], 31))) - 1).astype(np.uint32)), net).astype(np.uint32)
    plen = np.where(nest, np.maximum(plen, np.minimum(plen[parent] + rng.integers(1, 8, n_lpm), 31)), plen)
    mask = np.where(plen == 0, 0, (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF).astype(np.uint32)
    net = net & mask
    k, v = lpm_dedup(lpm4_keys(plen, net), np.ones((n_lpm, 1), np.uint8), 32)
    sc.add_map(MapSpec("cilium_cidr_v4_dyn", LPM, 8, 1, 65536, NO_PREALLOC, k, v))
    fix = rng.integers(0, 1 << 32, n_fix, dtype=np.uint64).astype(np.uint32)
    k, v = dedup(lpm4_keys(np.full(n_fix, 32), fix), np.ones((n_fix, 1), np.uint8))
    sc.add_map(MapSpec("cilium_cidr_v4_fix", HASH, 8, 1, 20971520, NO_PREALLOC, k, v))
    # v6 maps present (1% IPv6 traffic) with a few entries
    p6 = rand_v6(rng, 64)
    k6, v6 = lpm_dedup(lpm6_keys(np.full(64, 48), p6), np.ones((64, 1), np.uint8), 128)
    sc.add_map(MapSpec("cilium_cidr_v6_dyn", LPM, 20, 1, 65536, NO_PREALLOC, k6, v6))
    f6 = rand_v6(rng, 64)
    k6, v6 = dedup(lpm6_keys(np.full(64, 128), f6), np.ones((64, 1), np.uint8))
    sc.add_map(MapSpec("cilium_cidr_v6_fix", HASH, 20, 1, 20971520, NO_PREALLOC, k6, v6))
    # cilium_lxc: endpoints + 1 host entry
    ep = (ip4("10.1.0.0") + np.arange(1, n_ep + 1)).astype(np.uint32)
    ep6 = rand_v6(rng, 64, prefix=(0xf0, 0x0d))
    keys = np.concatenate([endpoint_keys4(ep), endpoint_keys4(np.array([ip4("10.0.0.1")], np.uint32)),
                           endpoint_keys6(ep6)])
    vals = endpoint_infos(np.concatenate([100 + np.arange(n_ep), [0], 100 + np.arange(64)]),
                          np.concatenate([np.full(n_ep, 256), [1], np.full(64, 256)]),
                          np.concatenate([1000 + np.arange(n_ep), [0], 3000 + np.arange(64)]),
                          np.concatenate([np.zeros(n_ep), [1], np.zeros(64)]).astype(np.uint32))
    sc.add_map(MapSpec("cilium_lxc", HASH, 20, 112, 65535, 0, keys, vals))
    sc.xdp = {"cidr4_hmap": "cilium_cidr_v4_fix", "cidr4_lmap": "cilium_cidr_v4_dyn",
              "cidr6_hmap": "cilium_cidr_v6_fix", "cidr6_lmap": "cilium_cidr_v6_dyn", "lxc_map": "cilium_lxc"}
    # packets: 97% v4, 1% v6, 1% ARP, 1% truncated
    n = n_packets
    kind = rng.random(n)
    is_v6 = (kind >= 0.97) & (kind < 0.98)
    is_arp = (kind >= 0.98) & (kind < 0.99)
    is_tr = kind >= 0.99
    s = rng.random(n)
    pick = rng.integers(0, len(net), n)
    inside = (net[pick] | (rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) &
                           ~mask[pick])).astype(np.uint32)
    saddr = np.where(s < 0.30, inside, np.where(s < 0.35, fix[rng.integers(0, n_fix, n)],
                                                rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)))
    daddr = np.where(rng.random(n) < 0.80, ep[rng.integers(0, n_ep, n)],
                     rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)).astype(np.uint32)
    proto = np.where(rng.random(n) < 0.7, TCP, UDP).astype(np.uint8)
    f, lens = frames_v4(n, stride, saddr, daddr, proto, rng.integers(1024, 65536, n), 80, F_ACK, payload=100)
    # IPv6 rows
    i6 = np.nonzero(is_v6)[0]
    if len(i6):
        s6 = np.where((rng.random(len(i6)) < 0.3)[:, None], f6[rng.integers(0, 64, len(i6))], rand_v6(rng, len(i6)))
        d6 = np.where((rng.random(len(i6)) < 0.8)[:, None], ep6[rng.integers(0, 64, len(i6))], rand_v6(rng, len(i6)))
        f6r, l6 = frames_v6(len(i6), stride, s6, d6, TCP, 40000, 443, F_ACK, payload=60)
        f[i6] = f6r
        lens[i6] = l6
    ia = np.nonzero(is_arp)[0]
    f[ia, 12], f[ia, 13] = 0x08, 0x06
    lens[ia] = 42
    it = np.nonzero(is_tr)[0]
    lens[it] = rng.integers(0, 34, len(it))
    sc.batches.append(Packets(f, lens.astype(np.uint32)))
    return sc


# ------------------------------------------------------------------ config 3: service LB
def lb4_population(rng, n_svc, vip_base):
    """Config 3's service population: n_svc frontends from vip_base
    (90% VIP:port, 10% L3-only), 1..19 backends each (mean 10) on 10.200/12, 30% on
    a port other than the frontend's; lbmap rows as AddSVC2BPFMap writes them
    (pkg/maps/lbmap/lbmap.go:320-371: slaves 1..count, then the master with count).
    Returns (vip, l3only, fport, revnat, keys, vals)."""
    vip = (vip_base + np.arange(n_svc)).astype(np.uint32)
    l3only = rng.random(n_svc) < 0.10
    ports = np.array([80, 443, 8080, 53, 6379, 5432, 9090, 3306, 8443, 11211], np.uint32)
    fport = np.where(l3only, 0, ports[rng.integers(0, len(ports), n_svc)]).astype(np.uint32)
    nbe = rng.integers(1, 20, n_svc)
    revnat = (np.arange(n_svc) % 65535 + 1).astype(np.uint32)
    svc_of_be = np.repeat(np.arange(n_svc), nbe)
    slave = np.concatenate([np.arange(1, c + 1) for c in nbe]) if n_svc <= 20000 else \
        (np.arange(len(svc_of_be)) - np.repeat(np.cumsum(nbe) - nbe, nbe) + 1)
    nb = len(svc_of_be)
    be_addr = (ip4("10.200.0.0") + rng.integers(0, 1 << 20, nb)).astype(np.uint32)
    diff = rng.random(nb) < 0.30
    be_port = np.where(diff, rng.integers(1024, 65536, nb), fport[svc_of_be]).astype(np.uint32)
    keys = np.concatenate([lb4_keys(vip[svc_of_be], fport[svc_of_be], slave), lb4_keys(vip, fport, np.zeros(n_svc))])
    vals = np.concatenate([lb4_vals(be_addr, be_port, np.zeros(nb), revnat[svc_of_be]),
                           lb4_vals(np.zeros(n_svc), np.zeros(n_svc), nbe, np.zeros(n_svc))])
    return vip, l3only, fport, revnat, keys, vals


def config3(n_packets=16_000_000, n_svc=100_000, seed=0xC1D40003, stride=64, max_entries=2_000_000,
            redirect=True):
    """BASELINE config 3 / SURVEY §8(d): bpf_lb.c, 100k services / ~1M backends."""
    rng = np.random.default_rng(seed)
    sc = Scenario("config3_lb")
    vip, l3only, fport, revnat, keys, vals = lb4_population(rng, n_svc, ip4("10.96.0.0"))
    sc.add_map(MapSpec("cilium_lb4_services", HASH, 8, 12, max_entries, 0, keys, vals))
    rk, rv = revnat4_entries(revnat, vip, fport)
    rk, rv = dedup(rk, rv)
    sc.add_map(MapSpec("cilium_lb4_reverse_nat", HASH, 2, 6, max_entries, 0, rk, rv))
    sc.lb = {"lb4": "cilium_lb4_services", "lb6": None,
             "flags": LB_L3 | LB_L4 | (LB_REDIRECT if redirect else 0), "redirect_ifindex": 1}
    n = n_packets
    u = rng.random(n)
    # Zipf(1.1) over services via inverse-CDF on ranks
    ranks = np.arange(1, n_svc + 1, dtype=np.float64)
    w = ranks ** -1.1
    cdf = np.cumsum(w) / w.sum()
    perm = rng.permutation(n_svc)
    svc = perm[np.minimum(np.searchsorted(cdf, rng.random(n)), n_svc - 1)]
    l3idx = np.nonzero(l3only)[0]
    svc_l3 = l3idx[rng.integers(0, len(l3idx), n)]
    daddr = np.where(u < 0.85, vip[svc], np.where(u < 0.90, vip[svc_l3],
                                                  rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)))
    dport = np.where(u < 0.85, np.where(fport[svc] == 0, rng.integers(1, 65536, n), fport[svc]),
                     rng.integers(1, 65536, n)).astype(np.uint32)
    proto = np.where(rng.random(n) < 0.8, TCP, UDP).astype(np.uint8)
    saddr = (ip4("10.1.0.0") + rng.integers(0, 1 << 16, n)).astype(np.uint32)
    sport = rng.integers(32768, 61000, n).astype(np.uint32)
    f, lens = frames_v4(n, stride, saddr, daddr.astype(np.uint32), proto, sport, dport, F_ACK, payload=200)
    fh = flow_hash(saddr, daddr, sport, dport, proto)
    sc.batches.append(Packets(f, lens, flow_hash=fh))
    return sc


# ------------------------------------------------------------------ config 2: bpf_lxc ingress
SERVICE_PORTS = np.array([80, 443, 8080, 53, 6379, 5432, 9090, 3306, 8443, 11211], np.uint32)


def _interleave(rng, n_flows, k, start_spread):
    """Order for k packets per flow: flow f's j-th packet lands in round s_f + j;
    rounds are concatenated and shuffled internally (per-flow order kept)."""
    s = rng.integers(0, start_spread, n_flows).astype(np.int64)
    rnd = (s[:, None] + np.arange(k)[None, :]).ravel()
    key = (rnd << np.int64(32)) | rng.integers(0, 1 << 31, n_flows * k).astype(np.int64)
    return np.argsort(key, kind="stable")


def config2_tables(n_pairs=1 << 20, n_ep=256, n_ids=4096, n_l3=2000, n_l4=4000, n_wc=32, n_cidr=128,
                   seed=0xC1D40002, ct_max=48_000_000, proxy_frac=0.10, now=100_000, cls_p=(0.45, 0.30, 0.15, 0.10)):
    """Tables of BASELINE config 2 (256 endpoints, 4k identities, per-endpoint
    policy/CIDR maps, global CT) and the address-pair population.  Returns
    (scenario, pairs, rng)."""
    rng = np.random.default_rng(seed)
    sc = Scenario("config2_ingress", now=now)
    ep_ip = (ip4("10.1.0.0") + 1 + np.arange(n_ep)).astype(np.uint32)
    lxc_id = (1000 + np.arange(n_ep)).astype(np.uint32)
    ifidx = (100 + np.arange(n_ep)).astype(np.uint32)
    user_ids = 256 + np.arange(n_ids)
    # ---- pairs
    pe = rng.integers(0, n_ep, n_pairs)
    cls = rng.choice(4, n_pairs, p=list(cls_p))                        # A: L3, B: L4, W: world/CIDR, D: deny
    pid = user_ids[rng.integers(0, n_ids, n_pairs)].astype(np.uint32)
    pid[cls == 2] = 2                                                   # WORLD_ID
    port1 = SERVICE_PORTS[rng.integers(0, len(SERVICE_PORTS), n_pairs)]
    port2 = SERVICE_PORTS[rng.integers(0, len(SERVICE_PORTS), n_pairs)]
    # per-endpoint CIDR prefixes inside 100.64.0.0/10 (/16../24)
    cplen = rng.integers(16, 25, (n_ep, n_cidr))
    cnet = (ip4("100.64.0.0") + rng.integers(0, 1 << 22, (n_ep, n_cidr))).astype(np.uint32)
    cmask = ((0xFFFFFFFF << (32 - cplen)) & 0xFFFFFFFF).astype(np.uint32)
    cnet &= cmask
    # remote addresses
    raddr = (ip4("10.128.0.0") + rng.integers(0, 1 << 23, n_pairs)).astype(np.uint32)
    w = cls == 2
    in_cidr = w & (rng.random(n_pairs) < 2 / 3)
    ci = rng.integers(0, n_cidr, n_pairs)
    host_bits = rng.integers(0, 1 << 32, n_pairs, dtype=np.uint64).astype(np.uint32)
    raddr = np.where(in_cidr, cnet[pe, ci] | (host_bits & ~cmask[pe, ci]), raddr)
    raddr = np.where(w & ~in_cidr, (ip4("198.18.0.0") + rng.integers(0, 1 << 17, n_pairs)).astype(np.uint32), raddr)
    raddr = raddr.astype(np.uint32)
    # ---- maps
    sc.add_map(MapSpec("cilium_ct4_global", LRU_HASH, 14, 48, ct_max, 0,
                       np.zeros((0, 14), np.uint8), np.zeros((0, 48), np.uint8)))
    revk, revv = revnat4_entries(np.arange(1, 257), (ip4("10.96.0.0") + np.arange(256)).astype(np.uint32),
                                 np.full(256, 80))
    sc.add_map(MapSpec("cilium_lb4_reverse_nat", HASH, 2, 6, 65536, 0, revk, revv))
    proxy_ep = rng.random(n_ep) < proxy_frac
    order = np.argsort(pe, kind="stable")
    bounds = np.searchsorted(pe[order], np.arange(n_ep + 1))
    for e in range(n_ep):
        mine = order[bounds[e]:bounds[e + 1]]
        a_ids = np.unique(pid[mine[cls[mine] == 0]])
        l3 = np.unique(np.concatenate([a_ids, user_ids[rng.integers(0, n_ids, max(0, n_l3 - len(a_ids)))]]))
        b = mine[cls[mine] == 1]
        fill = max(0, n_l4 - 2 * len(b))
        l4_id = np.concatenate([pid[b], pid[b], user_ids[rng.integers(0, n_ids, fill)]])
        l4_port = np.concatenate([port1[b], port1[b], SERVICE_PORTS[rng.integers(0, len(SERVICE_PORTS), fill)]])
        l4_proto = np.concatenate([np.full(len(b), TCP), np.full(len(b), UDP),
                                   np.where(rng.random(fill) < 0.7, TCP, UDP)])
        wc_port = np.concatenate([SERVICE_PORTS[rng.integers(0, len(SERVICE_PORTS), 2)],
                                  rng.integers(20000, 30000, max(0, n_wc - 2))])
        wc_proto = np.where(rng.random(len(wc_port)) < 0.7, TCP, UDP)
        proxy = np.zeros(len(l4_id), np.uint32)
        if proxy_ep[e]:
            proxy = np.where(l4_port == 443, 16000 + e, 0).astype(np.uint32)
        keys = np.concatenate([policy_keys(l4_id, l4_port, l4_proto), policy_keys(l3, np.zeros(len(l3)), np.zeros(len(l3))),
                               policy_keys(np.zeros(len(wc_port)), wc_port, wc_proto)])
        vals = np.concatenate([policy_vals(proxy), policy_vals(np.zeros(len(l3))), policy_vals(np.zeros(len(wc_port)))])
        keys, vals = dedup(keys, vals)
        pname = f"cilium_policy_{int(lxc_id[e])}"
        sc.add_map(MapSpec(pname, HASH, 8, 24, 16384, 0, keys, vals))
        ck, cv = lpm_dedup(lpm4_keys(cplen[e], cnet[e]), np.ones((n_cidr, 1), np.uint8), 32)
        cname = f"cilium_cidr4_ingress_{int(lxc_id[e])}"
        sc.add_map(MapSpec(cname, LPM, 8, 1, 16384, NO_PREALLOC, ck, cv))
        l4cfg = [(80, 15000 + e, TCP), (8080, 0, TCP)] if proxy_ep[e] else []
        sc.lxc.append({"lxc_id": int(lxc_id[e]), "seclabel": 256 + e, "policy": pname, "ct4": "cilium_ct4_global",
                       "ct6": None, "cidr4": cname, "cidr6": None, "revnat4": "cilium_lb4_reverse_nat",
                       "revnat6": None, "flags": LXC_PRODUCTION, "l4": l4cfg})
    pairs = dict(pe=pe, cls=cls, pid=pid, port1=port1, port2=port2, raddr=raddr, ep_ip=ep_ip, lxc_id=lxc_id,
                 ifidx=ifidx)
    return sc, pairs, rng


def config2(n_flows=16_777_216, n_pairs=1 << 20, n_ep=256, n_ids=4096, n_l3=2000, n_l4=4000, n_wc=32, n_cidr=128,
            pkts_per_flow=4, warm_frac=0.5, seed=0xC1D40002, stride=64, ct_max=48_000_000, proxy_frac=0.10,
            reply_frac=0.05, related_frac=0.01, unk_frac=0.005, trunc_frac=0.005, now=100_000):
    """BASELINE config 2 / SURVEY §8(d): bpf_lxc ingress, ct_lookup4 + policy.
    Host-generated frames (parity tests); the bench uses cilium_amd.stream."""
    sc, P, rng = config2_tables(n_pairs, n_ep, n_ids, n_l3, n_l4, n_wc, n_cidr, seed, ct_max, proxy_frac, now)
    pe, cls, pid, port1, port2, raddr = P["pe"], P["cls"], P["pid"], P["port1"], P["port2"], P["raddr"]
    ep_ip, lxc_id, ifidx = P["ep_ip"], P["lxc_id"], P["ifidx"]
    # ---- flows
    fp = rng.integers(0, n_pairs, n_flows)
    fe = pe[fp]
    u = rng.random(n_flows)
    proto = np.where(u < 0.70, TCP, np.where(u < 0.95, UDP, ICMP)).astype(np.uint8)
    sport = rng.integers(32768, 61000, n_flows).astype(np.uint32)
    dport = np.where(rng.random(n_flows) < 0.8, port1[fp], port2[fp]).astype(np.uint32)
    kind = rng.random(n_flows)
    is_reply = kind < reply_frac
    warm = (~is_reply) & (rng.random(n_flows) < warm_frac)
    # egress-created CT entries for reply flows (endpoint E:dport -> remote R:sport)
    ri = np.nonzero(is_reply & (proto != ICMP))[0]
    E, R = ep_ip[fe[ri]], raddr[fp[ri]]
    ctk = ct4_keys(E, R, raw16(sport[ri]), raw16(dport[ri]), proto[ri], np.zeros(len(ri)))
    relk = ct4_keys(E, R, np.zeros(len(ri)), np.zeros(len(ri)), np.full(len(ri), ICMP), np.full(len(ri), 2))
    revn = np.where(rng.random(len(ri)) < 0.2, raw16(rng.integers(1, 257, len(ri))), 0)
    ctv = ct_vals(len(ri), now + 43200, 16, 0, ep_ip[fe[ri]] & 0xffff, tx=(1, 100))
    ctv[:, 38:40] = le_bytes(revn, "<u2")
    relv = ct_vals(len(ri), now + 43200, 16, 0, 0, tx=(1, 100))
    k, v = dedup(np.concatenate([ctk, relk]), np.concatenate([ctv, relv]))
    sc.maps["cilium_ct4_global"].keys, sc.maps["cilium_ct4_global"].vals = k, v
    # ---- per-flow packet sequences
    K = pkts_per_flow
    nf = n_flows
    tcpf = np.zeros((nf, K), np.uint8)
    tcpf[:] = F_ACK
    tcpf[:, 0] = np.where(warm | is_reply, F_ACK, F_SYN)
    last = np.where(rng.random(nf) < 0.8, F_FIN | F_ACK, F_RST)
    tcpf[:, K - 1] = np.where(is_reply, F_ACK, last)
    icmpt = np.full((nf, K), 8, np.uint8)               # echo request
    rel = is_reply & (rng.random(nf) < related_frac / max(reply_frac, 1e-9))
    icmpt[rel, K - 1] = 3                                # DEST_UNREACH, related to the egress entry
    fproto = np.repeat(proto[:, None], K, axis=1)
    fproto[rel, K - 1] = ICMP
    # warm-up batch: first packet of warm flows
    wi = np.nonzero(warm)[0]
    wi = wi[rng.permutation(len(wi))]
    if len(wi):
        f, lens = frames_v4(len(wi), stride, raddr[fp[wi]], ep_ip[fe[wi]], proto[wi], sport[wi], dport[wi],
                            np.where(proto[wi] == TCP, F_SYN, 0), 8, payload=64)
        sc.batches.append(Packets(f, lens, pid[fp[wi]], ifidx[fe[wi]], lxc_id[fe[wi]].astype(np.uint16),
                                  np.zeros(len(wi), np.uint8)))
    # measured stream
    order = _interleave(rng, nf, K, max(1, K * 4))
    flow = order // K
    j = order % K
    n = len(order)
    pr = fproto[flow, j]
    s_ = np.where(is_reply[flow], raddr[fp[flow]], raddr[fp[flow]])
    f, lens = frames_v4(n, stride, s_, ep_ip[fe[flow]], pr, sport[flow], dport[flow], tcpf[flow, j],
                        icmpt[flow, j], payload=rng.integers(0, 1400, n))
    # unknown protocol / truncated packets
    x = rng.random(n)
    unk = x < unk_frac
    f[unk, 23] = 47
    tr = (x >= unk_frac) & (x < unk_frac + trunc_frac)
    lens = lens.copy()
    lens[tr] = rng.integers(14, 50, int(tr.sum()))
    tci = (rng.random(n) < 0.01).astype(np.uint8)     # a few packets from the egress proxy (skip proxy)
    sc.batches.append(Packets(f, lens.astype(np.uint32), pid[fp[flow]], ifidx[fe[flow]],
                              lxc_id[fe[flow]].astype(np.uint16), tci))
    sc.host_ifindex = 1
    sc.meta = {"n_flows": n_flows, "n_pairs": n_pairs, "n_ep": n_ep, "warm": int(warm.sum())}
    return sc


# ------------------------------------------------------------------ parity fuzz scenario
def fuzz(seed=1, n_packets=20000, n_batches=3, stride=128, ct_max=100000, ct6_max=100000):
    """Small shared pools so that map hits, repeated flows, replies, related
    ICMP, deletes, proxies, rev-NAT, weird IHL, truncation and IPv6
    extension-header chains all occur.  Used by the parity tests (a small
    ct_max / ct6_max makes the LRU CT maps overflow and exercises eviction)."""
    rng = np.random.default_rng(seed)
    sc = Scenario(f"fuzz{seed}", now=5000)
    n_ep = 16
    ep4 = (ip4("10.1.0.1") + np.arange(n_ep)).astype(np.uint32)
    ep6 = rand_v6(rng, n_ep, prefix=(0xf0, 0x0d, 0, 0, 0, 0, 0, 0))
    rem4 = np.concatenate([ip4("100.64.1.0") + rng.integers(0, 256, 12), ip4("100.64.2.0") + rng.integers(0, 256, 12),
                           ip4("10.128.0.0") + rng.integers(0, 1024, 16)]).astype(np.uint32)
    rem6 = rand_v6(rng, 24)
    rem6[:8, :6] = (0x20, 0x01, 0x0d, 0xb8, 0xaa, 0xbb)
    vip4 = (ip4("10.96.0.1") + np.arange(8)).astype(np.uint32)
    vip6 = rand_v6(rng, 8, prefix=(0xfd, 0x00))
    ports = np.array([80, 443, 53, 8080, 1000, 2000], np.uint32)
    lxc_id = (2000 + np.arange(n_ep)).astype(np.uint32)
    ids = np.concatenate([[1, 2, 3, 4], 256 + np.arange(24)]).astype(np.uint32)
    npool = 300
    pool = dict(s=rem4[rng.integers(0, len(rem4), npool)], ein=rng.integers(0, n_ep, npool),
                pr=rng.choice(np.array([TCP, TCP, UDP, ICMP], np.uint8), npool),
                sp=ports[rng.integers(0, len(ports), npool)], dp=ports[rng.integers(0, len(ports), npool)],
                sid=ids[rng.integers(0, len(ids), npool)])
    pool["pr"][:40] = np.where(rng.random(40) < 0.6, TCP, UDP)
    sc.meta["pool"] = pool
    sc.meta.update(ep6=ep6, rem6=rem6)

    # ---- XDP maps
    pl = np.array([24, 30, 16, 31, 8, 28, 25], np.uint32)
    nets = np.array([ip4("100.64.1.0"), ip4("100.64.2.4"), ip4("100.65.0.0"), ip4("100.64.2.128"),
                     ip4("44.0.0.0"), ip4("100.64.2.16"), ip4("10.128.1.0")], np.uint32)
    k, v = lpm_dedup(lpm4_keys(pl, nets), np.ones((len(pl), 1), np.uint8), 32)
    sc.add_map(MapSpec("v4_dyn", LPM, 8, 1, 1024, NO_PREALLOC, k, v))
    fix = rem4[rng.integers(0, len(rem4), 6)]
    k, v = dedup(lpm4_keys(np.full(6, 32), fix), np.ones((6, 1), np.uint8))
    sc.add_map(MapSpec("v4_fix", HASH, 8, 1, 1024, NO_PREALLOC, k, v))
    p6 = rem6[:4].copy()
    k, v = lpm_dedup(lpm6_keys(np.array([48, 64, 127, 128]), p6), np.ones((4, 1), np.uint8), 128)
    sc.add_map(MapSpec("v6_dyn", LPM, 20, 1, 1024, NO_PREALLOC, k, v))
    k, v = dedup(lpm6_keys(np.full(3, 128), rem6[10:13]), np.ones((3, 1), np.uint8))
    sc.add_map(MapSpec("v6_fix", HASH, 20, 1, 1024, NO_PREALLOC, k, v))
    lk = np.concatenate([endpoint_keys4(ep4[:12]), endpoint_keys6(ep6[:12])])
    lv = endpoint_infos(np.arange(24) + 10, np.full(24, 256), np.concatenate([lxc_id[:12], lxc_id[:12]]), np.zeros(24))
    sc.add_map(MapSpec("cilium_lxc", HASH, 20, 112, 65535, 0, lk, lv))
    sc.xdp = {"cidr4_hmap": "v4_fix", "cidr4_lmap": "v4_dyn", "cidr6_hmap": "v6_fix", "cidr6_lmap": "v6_dyn",
              "lxc_map": "cilium_lxc"}

    # ---- LB maps
    keys, vals = [], []
    for i, vip in enumerate(vip4):
        fp = 0 if i in (2, 5) else int(ports[i % len(ports)])
        cnt = int(rng.integers(1, 5))
        present = cnt if i != 3 else cnt - 1              # svc 3 misses its last slave -> DROP_NO_SERVICE
        mcount = 0 if i == 6 else cnt                      # svc 6 master has count 0 -> not a service
        keys.append(lb4_keys([vip], [fp], [0])); vals.append(lb4_vals([0], [0], [mcount], [0]))
        for s in range(1, present + 1):
            bp = fp if rng.random() < 0.6 else int(rng.integers(1, 65536))
            keys.append(lb4_keys([vip], [fp], [s]))
            vals.append(lb4_vals([ep4[rng.integers(0, n_ep)]], [bp], [0], [i + 1]))
    # an L3 fallback entry for a VIP that also has an L4 service
    keys.append(lb4_keys([vip4[0]], [0], [0])); vals.append(lb4_vals([0], [0], [2], [0]))
    for s in (1, 2):
        keys.append(lb4_keys([vip4[0]], [0], [s])); vals.append(lb4_vals([ep4[s]], [9000 + s], [0], [40]))
    k, v = dedup(np.concatenate(keys), np.concatenate(vals))
    sc.add_map(MapSpec("lb4_svc", HASH, 8, 12, 65536, 0, k, v))
    keys, vals = [], []
    for i in range(len(vip6)):
        fp = 0 if i == 2 else int(ports[i % len(ports)])
        cnt = int(rng.integers(1, 4))
        keys.append(lb6_keys(vip6[i:i + 1], [fp], [0])); vals.append(lb6_vals(np.zeros((1, 16), np.uint8), [0], [cnt], [0]))
        for s in range(1, cnt + 1):
            keys.append(lb6_keys(vip6[i:i + 1], [fp], [s]))
            vals.append(lb6_vals(ep6[rng.integers(0, n_ep)][None, :], [int(rng.integers(1, 65536))], [0],
                                 [int(rng.integers(0, 3))]))
    k, v = dedup(np.concatenate(keys), np.concatenate(vals))
    sc.add_map(MapSpec("lb6_svc", HASH, 20, 24, 65536, 0, k, v))
    sc.lb = {"lb4": "lb4_svc", "lb6": "lb6_svc", "flags": LB_L3 | LB_L4 | LB_REDIRECT, "redirect_ifindex": 1}

    # ---- ingress maps
    rk, rv = revnat4_entries(np.arange(1, 9), vip4, ports[np.arange(8) % len(ports)])
    rk2, rv2 = revnat4_entries([9, 10], vip4[:2], [0, 0])
    sc.add_map(MapSpec("revnat4", HASH, 2, 6, 65536, 0, np.concatenate([rk, rk2]), np.concatenate([rv, rv2])))
    rk, rv = revnat6_entries(np.arange(1, 4), vip6[:3], [80, 0, 443])
    sc.add_map(MapSpec("revnat6", HASH, 2, 18, 65536, 0, rk, rv))
    # CT maps pre-populated with egress-style entries (replies, related, closing, loopback, rev-NAT)
    npre = 40
    E, R = ep4[pool["ein"][:npre]], pool["s"][:npre]
    pr = pool["pr"][:npre]
    ek = ct4_keys(E, R, raw16(pool["sp"][:npre]), raw16(pool["dp"][:npre]), pr, np.zeros(npre))
    rel = ct4_keys(E, R, np.zeros(npre), np.zeros(npre), np.full(npre, ICMP), np.full(npre, 2))
    fl = rng.choice(np.array([0, 16, 1, 2, 3, 8, 24, 19], np.uint16), npre)
    rn = np.where(rng.random(npre) < 0.5, raw16(rng.integers(1, 12, npre)), 0).astype(np.uint16)
    ev = ct_vals(npre, 4000, 0, 0, 300, tx=(3, 300))
    ev[:, 36:38] = le_bytes(fl, "<u2")
    ev[:, 38:40] = le_bytes(rn, "<u2")
    k, v = dedup(np.concatenate([ek, rel]), np.concatenate([ev, ct_vals(npre, 4000, 16)]))
    sc.add_map(MapSpec("ct4", LRU_HASH, 14, 48, ct_max, 0, k, v))
    n6 = 12
    E6, R6 = ep6[rng.integers(0, n_ep, n6)], rem6[rng.integers(0, len(rem6), n6)]
    k6 = pack_rows(E6, R6, le_bytes(raw16(ports[rng.integers(0, len(ports), n6)]), "<u2"),
                   le_bytes(raw16(ports[rng.integers(0, len(ports), n6)]), "<u2"),
                   np.full((n6, 1), TCP, np.uint8), np.zeros((n6, 1), np.uint8), np.zeros((n6, 2), np.uint8))
    v6 = ct_vals(n6, 4000, 16, 0, 300)
    v6[:, 38:40] = le_bytes(np.where(rng.random(n6) < 0.5, raw16(rng.integers(1, 4, n6)), 0), "<u2")
    sc.add_map(MapSpec("ct6", LRU_HASH, 40, 48, ct6_max, 0, *dedup(k6, v6)))
    flag_sets = [LXC_PRODUCTION] * 10 + [LXC_PRODUCTION | LXC_DROP_ALL, LXC_PRODUCTION & ~LXC_POLICY_INGRESS,
                                         LXC_PRODUCTION & ~LXC_LXC_IPV4, LXC_PRODUCTION & ~LXC_HAVE_L4_POLICY,
                                         LXC_PRODUCTION & ~LXC_CT_ACCOUNTING, LXC_PRODUCTION]
    for e in range(n_ep):
        nl3, nl4, nwc = 8, 14, 3
        l3 = ids[rng.integers(0, len(ids), nl3)]
        l4i = ids[rng.integers(0, len(ids), nl4)]
        l4p = np.concatenate([ports[rng.integers(0, len(ports), nl4 - 2)], [8, 128]])   # ICMP echo "ports"
        l4x = np.concatenate([rng.choice([TCP, UDP], nl4 - 2), [ICMP, ICMPV6]])
        wcp = ports[rng.integers(0, len(ports), nwc)]
        wcx = rng.choice([TCP, UDP], nwc)
        proxy = np.where(rng.random(nl4) < 0.3, rng.integers(1, 65536, nl4), 0)
        kk = np.concatenate([policy_keys(l4i, l4p, l4x), policy_keys(l3, np.zeros(nl3), np.zeros(nl3)),
                             policy_keys(np.zeros(nwc), wcp, wcx)])
        vv = np.concatenate([policy_vals(proxy), policy_vals(np.zeros(nl3)),
                             policy_vals(np.where(rng.random(nwc) < 0.3, 7000, 0))])
        kk, vv = dedup(kk, vv)
        sc.add_map(MapSpec(f"pol{e}", HASH, 8, 24, 16384, 0, kk, vv))
        cp = np.array([24, 23, 28, 32], np.uint32)
        cn = np.array([ip4("100.64.1.0"), ip4("100.64.2.0"), rem4[rng.integers(0, 12)], rem4[rng.integers(0, 24)]],
                      np.uint32) & ((0xFFFFFFFF << (32 - cp)) & 0xFFFFFFFF).astype(np.uint32)
        ck, cv = lpm_dedup(lpm4_keys(cp[: 1 + e % 4], cn[: 1 + e % 4]), np.ones((1 + e % 4, 1), np.uint8), 32)
        sc.add_map(MapSpec(f"cidr4_{e}", LPM, 8, 1, 1024, NO_PREALLOC, ck, cv))
        ck6, cv6 = lpm_dedup(lpm6_keys(np.array([48, 128]), rem6[[0, 1 + e % 8]]), np.ones((2, 1), np.uint8), 128)
        sc.add_map(MapSpec(f"cidr6_{e}", LPM, 20, 1, 1024, NO_PREALLOC, ck6, cv6))
        l4cfg = [(80, 15000 + e, TCP), (53, 0, UDP), (443, 16000, UDP)] if e % 3 == 0 else []
        sc.lxc.append({"lxc_id": int(lxc_id[e]), "seclabel": 256 + e, "policy": f"pol{e}", "ct4": "ct4", "ct6": "ct6",
                       "cidr4": f"cidr4_{e}" if e != 5 else None, "cidr6": f"cidr6_{e}", "revnat4": "revnat4",
                       "revnat6": "revnat6", "flags": flag_sets[e], "l4": l4cfg})
    sc.host_ifindex = 3

    # ---- packets
    for bi in range(n_batches):
        n = n_packets
        kind = rng.random(n)
        v6m = (kind >= 0.80) & (kind < 0.93)
        oth = kind >= 0.97
        arp = (kind >= 0.93) & (kind < 0.97)
        # v4 fields
        to_vip = rng.random(n) < 0.25
        ein = rng.integers(0, n_ep, n)
        d4 = np.where(to_vip, vip4[rng.integers(0, 8, n)], ep4[ein])
        d4 = np.where(rng.random(n) < 0.05, rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32), d4)
        s4 = rem4[rng.integers(0, len(rem4), n)]
        rev = rng.random(n) < 0.15                       # reply direction from an endpoint
        s4, d4 = np.where(rev, d4, s4), np.where(rev, s4, d4)
        pr = rng.choice(np.array([TCP, TCP, TCP, UDP, UDP, ICMP, ICMP, ICMPV6, 47, 132], np.uint8), n)
        sp = ports[rng.integers(0, len(ports), n)]
        dp = ports[rng.integers(0, len(ports), n)]
        tf = np.where(rng.random(n) < 0.6, rng.choice(np.array([F_SYN, F_ACK, F_ACK, F_FIN | F_ACK, F_RST, F_SYN | F_ACK],
                                                               np.uint8), n), rng.integers(0, 256, n)).astype(np.uint8)
        it = rng.choice(np.array([0, 3, 8, 8, 11, 12, 5, 13, 1, 2, 4, 128, 129, 135], np.uint8), n)
        ihl = np.where(rng.random(n) < 0.08, rng.integers(0, 16, n), 5)
        # 60% of packets reuse a small pool of flows (both directions) so CT state builds up
        use = (rng.random(n) < 0.6) & ~to_vip
        pi = rng.integers(0, len(pool["s"]), n)
        ein = np.where(use, pool["ein"][pi], ein)
        s4 = np.where(use, np.where(rev, ep4[ein], pool["s"][pi]), s4)
        d4 = np.where(use, np.where(rev, pool["s"][pi], ep4[ein]), d4)
        pr = np.where(use, pool["pr"][pi], pr).astype(np.uint8)
        sp, dp = np.where(use, np.where(rev, pool["dp"][pi], pool["sp"][pi]), sp), \
            np.where(use, np.where(rev, pool["sp"][pi], pool["dp"][pi]), dp)
        it = np.where(use & (pr == ICMP), rng.choice(np.array([8, 8, 0, 3, 11], np.uint8), n), it).astype(np.uint8)
        f, lens = frames_v4(n, stride, s4, d4, pr, sp, dp, tf, it, 0, ihl, payload=rng.integers(0, 64, n))
        # IPv6 rows (with extension headers)
        i6 = np.nonzero(v6m)[0]
        m = len(i6)
        if m:
            de = np.where((rng.random(m) < 0.25)[:, None], vip6[rng.integers(0, 8, m)], ep6[rng.integers(0, n_ep, m)])
            se = rem6[rng.integers(0, len(rem6), m)]
            r6 = rng.random(m) < 0.15
            se, de = np.where(r6[:, None], de, se), np.where(r6[:, None], se, de)
            nh = rng.choice(np.array([TCP, TCP, UDP, ICMPV6, ICMPV6, ICMP, 47], np.uint8), m)
            ext = []
            depth = np.where(rng.random(m) < 0.25, rng.integers(1, 6, m), 0)
            for lvl in range(5):
                t = rng.choice(np.array([0, 60, 43, 51, 44, 59, 0], np.uint8), m)
                hl = rng.integers(0, 3, m).astype(np.uint8)
                ext.append((np.where(depth > lvl, t, 255).astype(np.uint8), hl))
            f6, l6 = frames_v6(m, stride, se, de, nh, sp[i6], dp[i6], tf[i6], it[i6], ext=ext,
                               payload=rng.integers(0, 64, m))
            f[i6] = f6
            lens[i6] = l6
        ia = np.nonzero(arp)[0]
        f[ia, 12], f[ia, 13] = 0x08, 0x06
        io = np.nonzero(oth)[0]
        f[io, 12], f[io, 13] = 0x88, 0xcc
        lens = lens.astype(np.int64)
        tr = rng.random(n) < 0.10
        lens[tr] = rng.integers(0, np.maximum(lens[tr], 1) + 1)
        lens = np.minimum(lens, stride + 400).astype(np.uint32)
        sid = np.where(use, pool["sid"][pi], ids[rng.integers(0, len(ids), n)]).astype(np.uint32)
        lid = np.where(rng.random(n) < 0.97, lxc_id[np.where(v6m, rng.integers(0, n_ep, n), ein)], 4242).astype(np.uint16)
        ifx = np.where(rng.random(n) < 0.9, 10 + ein, 0).astype(np.uint32)
        tci = (rng.random(n) < 0.1).astype(np.uint8)
        fh = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        sc.batches.append(Packets(f, lens, sid, ifx, lid, tci, fh))
    return sc


def conntrack_local(sc, every=1, max_entries=None):
    """The ConntrackLocal endpoint option (pkg/endpoint/bpf.go:268-276): every
    `every`-th endpoint of the scenario binds CT maps of its own,
    `<ct map>_<lxc_id>` (cilium_ct4_<id> / cilium_ct6_<id>), created like the map
    it had (type, sizes, the prefilled entries copied), with `max_entries` if given;
    the other endpoints keep the shared ones.  Returns the new map names."""
    made = []
    for j, e in enumerate(sc.lxc):
        if j % every:
            continue
        for fam in ("ct4", "ct6"):
            name = e.get(fam)
            if not name:
                continue
            src = sc.maps[name]
            local = f"{name}_{e['lxc_id']}"
            keys = None if src.keys is None else src.keys.copy()
            vals = None if src.vals is None else src.vals.copy()
            if max_entries is not None and keys is not None and len(keys) > max_entries:
                keys, vals = keys[:max_entries], vals[:max_entries]
            sc.add_map(MapSpec(local, src.type, src.ksz, src.vsz, max_entries or src.max_entries, src.flags, keys, vals))
            e[fam] = local
            made.append(local)
    return made


def pipeline_fuzz(seed=3, n_packets=20000, n_batches=3, lb_redirect=False, fixed_secctx=None, proxy_max=524288):
    """The fuzz scenario run through the whole pipeline (bpf_xdp -> bpf_lb ->
    bpf_netdev -> handle_policy): endpoint MACs and port maps (duplicated and
    unterminated entries), host endpoints, VIPs present in cilium_lxc as host
    entries (so the prefilter passes them), TTL / hop-limit 0..1, random IPv4
    and L4 checksums (UDP 0 = no checksum), sources inside ROUTER_IP/64.
    256-B snaps hold every header byte the programs touch."""
    sc = fuzz(seed, n_packets, n_batches, stride=256)
    sc.name = f"pipe{seed}"
    rng = np.random.default_rng(seed ^ 0x5151)
    lxc = sc.maps["cilium_lxc"]
    n = lxc.n()
    v = lxc.vals.copy()
    v[:, 16:22] = rng.integers(0, 256, (n, 6))
    v[:, 24:30] = rng.integers(0, 256, (n, 6))
    ports = np.array([80, 443, 53, 8080, 1000, 2000], np.uint32)
    for e in range(n):
        if e % 3 == 1:
            k = int(rng.integers(1, 6))
            frm = ports[rng.integers(0, len(ports), k)]
            to = rng.integers(1, 65536, k)
            if e % 2:
                frm[-1] = frm[0]                        # two entries for one port: both apply
            pm = np.stack([raw16(frm), raw16(to)], axis=1).astype("<u2").view(np.uint8).reshape(-1)
            v[e, 48:48 + 4 * k] = pm
            if e == 4:
                v[e, 48 + 4 * k:48 + 4 * k + 2] = 1     # a 'from' without 'to' ends the list
    v[3, 8:12] = 1                                      # ENDPOINT_F_HOST (v4)
    v[15, 8:12] = 1                                     # ENDPOINT_F_HOST (v6)
    # VIPs as host entries (half of them), so bpf_xdp's endpoint check passes them
    vip4 = (ip4("10.96.0.1") + np.arange(8)).astype(np.uint32)[::2]
    hk = endpoint_keys4(vip4)
    hv = endpoint_infos(np.full(len(vip4), 1), np.zeros(len(vip4)), np.zeros(len(vip4)), np.ones(len(vip4)))
    lb6 = sc.maps["lb6_svc"]
    vip6 = np.unique(lb6.keys[:, :16], axis=0)[::2]
    hk6 = endpoint_keys6(vip6)
    hv6 = endpoint_infos(np.full(len(vip6), 1), np.zeros(len(vip6)), np.zeros(len(vip6)), np.ones(len(vip6)))
    lxc.keys, lxc.vals = dedup(np.concatenate([lxc.keys, hk, hk6]), np.concatenate([v, hv, hv6]))
    router = np.zeros(16, np.uint8)
    router[:8] = (0x20, 0x01, 0x0d, 0xb8, 0xaa, 0xbb, 0, 0)
    for pk in sc.batches:
        f = pk.frames
        m = pk.n
        et = (f[:, 12].astype(np.uint32) << 8) | f[:, 13]
        ttl = np.where(rng.random(m) < 0.06, rng.integers(0, 2, m), rng.integers(2, 256, m)).astype(np.uint8)
        v4 = et == 0x0800
        v6 = et == 0x86DD
        f[v4, 22] = ttl[v4]
        f[v6, 21] = ttl[v6]
        f[v4, 24:26] = rng.integers(0, 256, (int(v4.sum()), 2))
        # L4 checksum fields (TCP +16, UDP +6 after an IHL-derived offset), 10% zero
        l4 = 14 + (f[:, 14] & 0xf).astype(np.int64) * 4
        pr = f[:, 23]
        off = np.where(pr == 6, l4 + 16, np.where(pr == 17, l4 + 6, -1))
        ck = rng.integers(0, 65536, m)
        ck[rng.random(m) < 0.1] = 0
        ok = v4 & (off >= 0) & (off + 1 < f.shape[1])
        rows = np.nonzero(ok)[0]
        f[rows, off[ok]] = (ck[ok] >> 8).astype(np.uint8)
        f[rows, off[ok] + 1] = (ck[ok] & 0xff).astype(np.uint8)
        # IPv6 sources inside ROUTER_IP/64 (derive_sec_ctx takes the flow label)
        r6 = np.nonzero(v6 & (rng.random(m) < 0.2))[0]
        f[r6, 22:30] = router[:8]
        f[r6, 15:18] = rng.integers(0, 256, (len(r6), 3))
    if not lb_redirect:
        sc.lb = dict(sc.lb, flags=LB_L3 | LB_L4)
    sc.netdev = {"lxc_map": "cilium_lxc", "flags": 0 if fixed_secctx is None else 1,
                 "fixed_secctx": fixed_secctx or 0, "router_ip6": bytes(router)}
    # cilium_proxy4/6 (bpf/lib/maps.h:56-71; key 10 / 22 B, value 16 / 28 B) and the
    # node_config.h addresses of the proxy redirect (IPV4_GATEWAY, HOST_IP, MACs)
    sc.add_map(MapSpec("cilium_proxy4", HASH, 10, 16, proxy_max, 0))
    sc.add_map(MapSpec("cilium_proxy6", HASH, 22, 28, proxy_max, 0))
    sc.node = {"proxy4": "cilium_proxy4", "proxy6": "cilium_proxy6", "ipv4_gateway": 0xfffff50a,
               "host_ip6": bytes([0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0xa, 0, 0x2, 0xf, 0xff, 0xff]),
               "host_mac": bytes([0xce, 0x72, 0xa7, 0x03, 0x88, 0x56]),
               "node_mac": bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])}
    return sc


# ------------------------------------------------------------------ config 4: full pipeline tables
def config4_tables(n_pairs=1 << 20, n_lpm=10_000, n_fix=2_000, ct_max=64_000_000, seed=0xC1D40004,
                   n_svc=100_000, **kw):
    """BASELINE config 4 / SURVEY §8(d): the tables of configs 1-3 on one node,
    composed as bpf_xdp -> bpf_lb -> bpf_netdev -> handle_policy.  Config 2's
    endpoints/policies/CT; config 1's prefilter (10k LPM prefixes + 2k /32s);
    a service VIP per endpoint for each of SERVICE_PORTS (one backend: the
    endpoint itself, 30% on another port), present in cilium_lxc as host
    entries so the prefilter's endpoint check passes them; and config 3's
    service population (n_svc services / ~10 x n_svc backends on 10.98/15, the
    traffic's lookups probe the same 2M-entry lbmap).  Returns
    (scenario, pairs, vip_ip[n_ep])."""
    # traffic arriving on the netdev carries WORLD_ID (derive_ipv4_sec_ctx, bpf_netdev.c:249-261):
    # most pairs are world peers, admitted by the endpoints' CIDR / L4-wildcard rules
    kw.setdefault("cls_p", (0.05, 0.10, 0.75, 0.10))
    sc, P, rng = config2_tables(n_pairs=n_pairs, ct_max=ct_max, **kw)
    rng4 = np.random.default_rng(seed)
    n_ep = len(P["ep_ip"])
    # prefilter: prefixes outside the pair populations' ranges except for a few
    u = rng4.random(n_lpm)
    plen = np.where(u < 0.55, 24, np.where(u < 0.85, rng4.integers(16, 24, n_lpm), rng4.integers(25, 32, n_lpm)))
    net = (ip4("20.0.0.0") + rng4.integers(0, 1 << 28, n_lpm)).astype(np.uint32)
    hit = rng4.random(n_lpm) < 0.02                     # ~2% of prefixes cover pair addresses
    net = np.where(hit, P["raddr"][rng4.integers(0, n_pairs, n_lpm)], net).astype(np.uint32)
    mask = ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF).astype(np.uint32)
    k, v = lpm_dedup(lpm4_keys(plen, net & mask), np.ones((n_lpm, 1), np.uint8), 32)
    sc.add_map(MapSpec("cilium_cidr_v4_dyn", LPM, 8, 1, 65536, NO_PREALLOC, k, v))
    fix = np.concatenate([(ip4("20.0.0.0") + rng4.integers(0, 1 << 28, n_fix - 64)).astype(np.uint32),
                          P["raddr"][rng4.integers(0, n_pairs, 64)]])
    k, v = dedup(lpm4_keys(np.full(n_fix, 32), fix), np.ones((n_fix, 1), np.uint8))
    sc.add_map(MapSpec("cilium_cidr_v4_fix", HASH, 8, 1, 20971520, NO_PREALLOC, k, v))
    vip = (ip4("10.96.0.0") + 1 + np.arange(n_ep)).astype(np.uint32)
    keys = np.concatenate([endpoint_keys4(P["ep_ip"]), endpoint_keys4(vip)])
    vals = endpoint_infos(np.concatenate([P["ifidx"], np.zeros(n_ep)]),
                          np.concatenate([256 + np.arange(n_ep), np.ones(n_ep)]),
                          np.concatenate([P["lxc_id"], np.zeros(n_ep)]),
                          np.concatenate([np.zeros(n_ep), np.ones(n_ep)]).astype(np.uint32))
    vals[:n_ep, 16:22] = rng4.integers(0, 256, (n_ep, 6))
    vals[:n_ep, 24:30] = rng4.integers(0, 256, (n_ep, 6))
    sc.add_map(MapSpec("cilium_lxc", HASH, 20, 112, 65535, 0, keys, vals))
    sp = SERVICE_PORTS
    ns = n_ep * len(sp)
    sv_vip = np.repeat(vip, len(sp))
    sv_port = np.tile(sp, n_ep)
    sv_ep = np.repeat(P["ep_ip"], len(sp))
    be_port = np.where(rng4.random(ns) < 0.3, np.roll(sv_port, 1), sv_port).astype(np.uint32)
    keys = np.concatenate([lb4_keys(sv_vip, sv_port, np.zeros(ns)), lb4_keys(sv_vip, sv_port, np.ones(ns))])
    vals = np.concatenate([lb4_vals(np.zeros(ns), np.zeros(ns), np.ones(ns), np.zeros(ns)),
                           lb4_vals(sv_ep, be_port, np.zeros(ns), (np.arange(ns) % 256) + 1)])
    if n_svc:
        _, _, _, _, k3, v3 = lb4_population(np.random.default_rng(seed + 3), n_svc, ip4("10.98.0.0"))
        keys, vals = np.concatenate([keys, k3]), np.concatenate([vals, v3])
    sc.add_map(MapSpec("cilium_lb4_services", HASH, 8, 12, 2_000_000, 0, keys, vals))
    sc.xdp = {"cidr4_hmap": "cilium_cidr_v4_fix", "cidr4_lmap": "cilium_cidr_v4_dyn", "cidr6_hmap": None,
              "cidr6_lmap": None, "lxc_map": "cilium_lxc"}
    sc.lb = {"lb4": "cilium_lb4_services", "lb6": None, "flags": LB_L3 | LB_L4, "redirect_ifindex": 0}
    sc.netdev = {"lxc_map": "cilium_lxc", "flags": 0}
    sc.name = "config4_pipeline"
    return sc, P, vip


# ------------------------------------------------------------------ config 5: IPv6 pipeline
ROUTER6 = bytes([0x20, 0x01, 0x0d, 0xb8, 0xaa, 0xaa, 0xbb, 0xbb, 0, 0, 0, 0, 0, 0, 0, 1])   # ROUTER_IP
NAT64 = bytes([0x00, 0x64, 0xff, 0x9b] + [0] * 12)                                        # 64:ff9b::/96


def v6_embed(prefix16, v4):
    """Addresses prefix16[:12] + the IPv4 address (host order) in bytes 12..15."""
    v4 = np.asarray(v4, np.uint32)
    a = np.tile(np.frombuffer(bytes(prefix16), np.uint8), (len(v4), 1))
    a[:, 12:16] = be32_bytes(v4)
    return a


def config5_tables(n_pairs=1 << 20, prefill=8_000_000, n_fix=100_000, n_dyn=10_000, ct6_max=10_485_760,
                   seed=0xC1D40005, now=100_000, reply_steps=16, flows_per_step=1 << 20):
    """BASELINE config 5 / SURVEY §8(d): the IPv6 path a packet takes on a node —
    bpf_xdp check_v6 (v6_dyn LPM: n_dyn prefixes /32-/127; v6_fix hash: n_fix
    /128s; cilium_lxc endpoint check) -> bpf_netdev handle_ipv6 (the identity of a
    source inside ROUTER_IP's /64 is its flow label, others are WORLD) ->
    handle_policy / ipv6_policy (ct_lookup6 on cilium_ct6_global, max_entries
    ct6_max, LRU, pre-filled to `prefill` entries: egress-created reply entries of
    the stream's reply flows plus older unrelated connections, 20% of them
    closing).  Endpoints, identities and per-endpoint policy are config 2's; the
    pairs' remote addresses become cluster sources (identity classes) or NAT64
    world sources (CIDR class, per-endpoint v6 CIDR maps of the same prefixes).
    Returns (scenario, pairs, meta)."""
    sc, P, rng = config2_tables(n_pairs=n_pairs, ct_max=1 << 16, seed=0xC1D40002, now=now)
    rng5 = np.random.default_rng(seed)
    sc.name = "config5_ipv6"
    n_ep = len(P["ep_ip"])
    ep6 = np.zeros((n_ep, 16), np.uint8)
    ep6[:, 0:2] = (0xfd, 0x00)
    ep6[:, 8:10] = (0x0a, 0x01)                      # bytes 12-13 zero: no rev-NAT index (bpf_lxc.c:776)
    ep6[:, 14:16] = be16_bytes(1 + np.arange(n_ep))
    world = P["cls"] == 2
    src6 = np.where(world[:, None], v6_embed(NAT64, P["raddr"]), v6_embed(ROUTER6[:8] + bytes(8), P["raddr"]))
    dst6 = ep6[P["pe"]]
    # per-endpoint v6 CIDR ingress maps: the v4 prefixes of config 2 under 64:ff9b::/96
    crng = np.random.default_rng(0xC1D40002 ^ 0x66)
    for e, cfg in enumerate(sc.lxc):
        k4 = sc.maps[cfg["cidr4"]].keys
        plen = k4[:, 0:4].copy().view("<u4").ravel()
        net = k4[:, 4:8].copy().view(">u4").ravel()
        ck, cv = lpm_dedup(lpm6_keys(96 + plen, v6_embed(NAT64, net)), np.ones((len(plen), 1), np.uint8), 128)
        name = f"cilium_cidr6_ingress_{cfg['lxc_id']}"
        sc.add_map(MapSpec(name, LPM, 20, 1, 16384, NO_PREALLOC, ck, cv))
        cfg.update(ct6="cilium_ct6_global", cidr6=name, revnat6="cilium_lb6_reverse_nat")
    rk, rv = revnat6_entries(np.arange(1, 257), v6_embed(bytes([0xfd, 0, 0, 0, 0, 0, 0, 0, 0, 0x60] + [0] * 6),
                                                        np.arange(256)), np.full(256, 80))
    sc.add_map(MapSpec("cilium_lb6_reverse_nat", HASH, 2, 18, 65536, 0, rk, rv))
    # cilium_lxc: the endpoints' IPv6 addresses (family 2) with their MACs
    ev = endpoint_infos(P["ifidx"], 256 + np.arange(n_ep), P["lxc_id"], np.zeros(n_ep))
    ev[:, 16:22] = rng5.integers(0, 256, (n_ep, 6))
    ev[:, 24:30] = rng5.integers(0, 256, (n_ep, 6))
    sc.add_map(MapSpec("cilium_lxc", HASH, 20, 112, 65535, 0, endpoint_keys6(ep6), ev))
    # prefilter: v6_fix /128s and v6_dyn /32-/127 prefixes (sized with the CIDR4 constants, bpf_xdp.c:73,83)
    fx = rand_v6(rng5, n_fix, prefix=(0x20, 0x01, 0x0d, 0xb8, 0xf0))
    hit = rng5.integers(0, n_pairs, 64)
    fx[:64] = src6[hit]
    k, v = dedup(lpm6_keys(np.full(n_fix, 128), fx), np.ones((n_fix, 1), np.uint8))
    sc.add_map(MapSpec("cilium_cidr_v6_fix", HASH, 20, 1, 20971520, NO_PREALLOC, k, v))
    dl = rng5.integers(32, 128, n_dyn)
    dn = rand_v6(rng5, n_dyn, prefix=(0x2a,))          # 2a00::/8: disjoint from the sources' /32s
    cov = rng5.random(n_dyn) < 0.02                  # a few prefixes cover pair sources
    dn[cov] = src6[rng5.integers(0, n_pairs, int(cov.sum()))]
    dl = np.where(cov, rng5.integers(120, 128, n_dyn), dl)
    k, v = lpm_dedup(lpm6_keys(dl, dn), np.ones((n_dyn, 1), np.uint8), 128)
    sc.add_map(MapSpec("cilium_cidr_v6_dyn", LPM, 20, 1, 65536, NO_PREALLOC, k, v))
    sc.xdp = {"cidr4_hmap": None, "cidr4_lmap": None, "cidr6_hmap": "cilium_cidr_v6_fix",
              "cidr6_lmap": "cilium_cidr_v6_dyn", "lxc_map": "cilium_lxc"}
    sc.lb = None
    sc.netdev = {"lxc_map": "cilium_lxc", "flags": 0, "router_ip6": ROUTER6}
    sc.add_map(MapSpec("cilium_ct6_global", LRU_HASH, 40, 48, ct6_max, 0))
    meta = dict(ep6=ep6, src6=src6, dst6=dst6, prefill=prefill, reply_steps=reply_steps,
                flows_per_step=flows_per_step)
    return sc, P, meta


def ct6_keys(d16, s16, dport_raw, sport_raw, nexthdr, flags):
    n = len(d16)
    return pack_rows(np.asarray(d16, np.uint8), np.asarray(s16, np.uint8), le_bytes(dport_raw, "<u2"),
                     le_bytes(sport_raw, "<u2"), np.asarray(nexthdr, np.uint8).reshape(n, 1),
                     np.asarray(flags, np.uint8).reshape(n, 1), np.zeros((n, 2), np.uint8))


def ct6_prefill(meta, reply_keys, reply_vals, now, seed=0xC1D40055):
    """cilium_ct6_global's pre-population: the reply flows' egress entries plus
    older connections of unrelated remote peers up to meta['prefill'] entries
    (lifetimes spread over the last 11 hours, 20% closing with short lifetimes)."""
    rng = np.random.default_rng(seed)
    n = max(0, meta["prefill"] - len(reply_keys))
    E = meta["ep6"][rng.integers(0, len(meta["ep6"]), n)]
    R = rand_v6(rng, n, prefix=(0x20, 0x01, 0x0d, 0xb8, 0x50, 0x00))
    pr = np.where(rng.random(n) < 0.7, TCP, UDP).astype(np.uint8)
    k = ct6_keys(E, R, raw16(rng.integers(1024, 65536, n)), raw16(rng.integers(1, 65536, n)), pr,
                 rng.integers(0, 2, n))
    closing = rng.random(n) < 0.2
    life = np.where(closing, now - rng.integers(0, 600, n) + 10, now - rng.integers(0, 40000, n) + 43200)
    v = ct_vals(n, 0, 0, 0, 0, rx=(3, 300), tx=(2, 200))
    v[:, 32:36] = le_bytes(life.astype(np.uint32), "<u4")
    v[:, 36:38] = le_bytes(np.where(closing, 3, 16).astype(np.uint16), "<u2")
    v[:, 44:48] = le_bytes(rng.integers(256, 4352, n).astype(np.uint32), "<u4")
    return dedup(np.concatenate([reply_keys, k]), np.concatenate([reply_vals, v]))


# ------------------------------------------------------------------ endpoint egress (from-container)
LXC_POLICY_EGRESS = 32
LXC_TRACE_NOTIFY = 64          # TRACE_NOTIFY (pkg/endpoint/endpoint.go:131-134)
NETDEV_TRACE_NOTIFY = 2


def egress_fuzz(seed=5, n_packets=20000, n_batches=3, proxy_max=524288, hazard=True, icmp=True):
    """Frames sent by the local endpoints through their from-container program
    (bpf_lxc.c handle_ingress -> handle_ipv4_from_lxc): services whose backends
    are local endpoints (local delivery after lb4_local, loopback back to the
    sender), remote peers behind the tunnel map, cluster and world peers, host
    entries, source-MAC / gateway-MAC / source-IP violations, port maps,
    POLICY_EGRESS endpoints with ipcache identities and egress CIDR maps,
    pre-populated reply / related / loopback CT entries (egress rev-NAT), a
    shared flow pool so that CT state builds up across the batches, and the
    pipeline's TTL / checksum randomisation.  Local deliveries continue into
    handle_policy of the destination endpoint.  hazard=False leaves out the
    tuples that make a batch run as a single bucket (an endpoint sending to
    itself, IPV4_LOOPBACK as a destination), so the parallel schedule and the
    deferred service entries are exercised."""
    sc = pipeline_fuzz(seed, n_packets=8, n_batches=1, proxy_max=proxy_max)
    sc.name = f"egress{seed}"
    sc.batches = []
    rng = np.random.default_rng(seed ^ 0xE6E5)
    n_ep = 16
    ep4 = (ip4("10.1.0.1") + np.arange(n_ep)).astype(np.uint32)
    lxc_id = (2000 + np.arange(n_ep)).astype(np.uint32)
    vip4 = (ip4("10.96.0.1") + np.arange(8)).astype(np.uint32)
    rem4 = np.concatenate([ip4("100.64.1.0") + rng.integers(0, 256, 12), ip4("10.128.0.0") + rng.integers(0, 1024, 12),
                           ip4("10.200.0.0") + rng.integers(0, 256, 8)]).astype(np.uint32)
    ports = np.array([80, 443, 53, 8080, 1000, 2000], np.uint32)
    node_mac = bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])
    macs = rng.integers(0, 256, (n_ep, 6)).astype(np.uint8)
    # ipcache (identities of remote peers), tunnel map (remote node prefixes), egress CIDR maps
    ic_ip = np.concatenate([rem4[:6], rem4[12:16], ep4[:4]])
    ic_id = np.concatenate([rng.integers(256, 280, 6), [2, 3, 2, 300], 256 + np.arange(4)]).astype(np.uint32)
    icv = np.zeros((len(ic_ip), 8), np.uint8)
    icv[:, 0:2] = le_bytes(ic_id, "<u2")
    sc.add_map(MapSpec("cilium_ipcache", HASH, 20, 8, 512000, 0, *dedup(endpoint_keys4(ic_ip), icv)))
    tk = endpoint_keys4(np.array([ip4("10.128.0.0"), ip4("10.200.0.0")], np.uint32))
    tv = endpoint_keys4(np.array([ip4("192.168.7.2"), ip4("192.168.7.3")], np.uint32))
    sc.add_map(MapSpec("cilium_tunnel_map", HASH, 20, 20, 65536, 0, tk, tv))
    # egress policy entries (key.egress = 1) in every endpoint's policy map
    ids = np.concatenate([[1, 2, 3, 4], 256 + np.arange(24)]).astype(np.uint32)
    for e in range(n_ep):
        m = sc.maps[f"pol{e}"]
        nl3, nl4, nwc = 6, 10, 3
        l3 = ids[rng.integers(0, len(ids), nl3)]
        l4i = ids[rng.integers(0, len(ids), nl4)]
        l4p = ports[rng.integers(0, len(ports), nl4)]
        l4x = rng.choice([TCP, UDP], nl4)
        proxy = np.where(rng.random(nl4) < 0.3, rng.integers(1, 65536, nl4), 0)
        kk = np.concatenate([m.keys, policy_keys(l4i, l4p, l4x, 1), policy_keys(l3, np.zeros(nl3), np.zeros(nl3), 1),
                             policy_keys(np.zeros(nwc), ports[rng.integers(0, len(ports), nwc)],
                                         rng.choice([TCP, UDP], nwc), 1)])
        vv = np.concatenate([m.vals, policy_vals(proxy), policy_vals(np.zeros(nl3)), policy_vals(np.zeros(nwc))])
        m.keys, m.vals = dedup(kk, vv)
        if e % 2 == 0:
            cp = np.array([16, 24, 32], np.uint32)
            cn = np.array([ip4("100.64.0.0"), rem4[12] & 0xFFFFFF00, rem4[20]], np.uint32)
            ck, cv = lpm_dedup(lpm4_keys(cp[: 1 + e % 3], cn[: 1 + e % 3]), np.ones((1 + e % 3, 1), np.uint8), 32)
            sc.add_map(MapSpec(f"cidr4e_{e}", LPM, 8, 1, 1024, NO_PREALLOC, ck, cv))
    ep6, rem6 = sc.meta["ep6"], sc.meta["rem6"]
    vip6 = np.unique(sc.maps["lb6_svc"].keys[:, :16], axis=0)
    router6 = bytes([0x20, 0x01, 0x0d, 0xb8, 0xaa, 0xbb, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1])
    for e in range(n_ep):
        if e % 2 == 1:
            ck6, cv6 = lpm_dedup(lpm6_keys(np.array([32, 128]), rem6[[0, 5 + e % 8]]), np.ones((2, 1), np.uint8), 128)
            sc.add_map(MapSpec(f"cidr6e_{e}", LPM, 20, 1, 1024, NO_PREALLOC, ck6, cv6))
    ic6 = np.concatenate([rem6[:5], ep6[:3]])
    icv6 = np.zeros((len(ic6), 8), np.uint8)
    icv6[:, 0:2] = le_bytes(np.concatenate([rng.integers(256, 280, 4), [2], 256 + np.arange(3)]), "<u2")
    ipc = sc.maps["cilium_ipcache"]
    ipc.keys, ipc.vals = dedup(np.concatenate([ipc.keys, endpoint_keys6(ic6)]), np.concatenate([ipc.vals, icv6]))
    tk6 = np.zeros((1, 20), np.uint8)
    tk6[0, :12] = rem6[7][:12]
    tk6[0, 16] = 2
    tm = sc.maps["cilium_tunnel_map"]
    tm.keys, tm.vals = np.concatenate([tm.keys, tk6]), np.concatenate([tm.vals, endpoint_keys4(np.array([ip4("192.168.7.9")], np.uint32))])
    for e, cfg in enumerate(sc.lxc):
        cfg["lxc_ip6"] = bytes(ep6[e])
        cfg["lb6"] = "lb6_svc" if e != 9 else None
        if e % 2 == 1 and e % 4 in (1, 2):
            cfg["cidr6e"] = f"cidr6e_{e}"
        cfg["lxc_mac"] = bytes(macs[e])
        cfg["node_mac"] = node_mac if e != 7 else bytes(6)
        cfg["lxc_ipv4"] = int(be32_bytes([ep4[e]]).view("<u4")[0, 0])
        cfg["lb4"] = "lb4_svc" if e != 9 else None
        cfg["ipcache"] = "cilium_ipcache"
        if e % 4 in (1, 2):
            cfg["flags"] |= LXC_POLICY_EGRESS
            cfg["cidr4e"] = f"cidr4e_{e}" if e % 2 == 0 else None
        if e % 5 == 2:
            cfg["portmap"] = [(30000 + e, 80), (30100 + e, 53)] + ([(30200, 80)] if e == 2 else [])
        if e % 3 == 1:
            cfg["l4e"] = [(80, 17000 + e, TCP), (53, 0, UDP), (443, 18000, TCP)]
    raw_be = lambda a: int(be32_bytes([a]).view("<u4")[0, 0])
    sc.node = dict(sc.node, lxc_map="cilium_lxc", ipv4_cluster_range=raw_be(ip4("10.0.0.0")),
                   ipv4_cluster_mask=raw_be(0xFF000000), ipv4_loopback=raw_be(ip4("10.255.255.245")),
                   ipv4_mask=raw_be(0xFFFF0000), encap_ifindex=5, tunnel_map="cilium_tunnel_map", router_ip6=router6)
    # CT entries the egress path meets as replies / related (rev-NAT, loopback) and as established flows
    ct = sc.maps["ct4"]
    npre = 48
    E = ep4[rng.integers(0, n_ep, npre)]
    R = np.where(rng.random(npre) < 0.5, rem4[rng.integers(0, len(rem4), npre)], ep4[rng.integers(0, n_ep, npre)])
    if not hazard:
        R = np.where(R == E, rem4[0], R)
    a, b = ports[rng.integers(0, len(ports), npre)], ports[rng.integers(0, len(ports), npre)]
    pr = rng.choice(np.array([TCP, TCP, UDP, ICMP], np.uint8), npre)
    rk = ct4_keys(R, E, raw16(a), raw16(b), pr, np.ones(npre))                 # egress REPLY probe key
    relk = ct4_keys(R, E, np.zeros(npre), np.zeros(npre), np.full(npre, ICMP), np.full(npre, 3))
    estk = ct4_keys(E, R, raw16(b), raw16(a), pr, np.zeros(npre))             # egress forward key
    fl = rng.choice(np.array([0, 16, 1, 2, 3, 8, 24, 19], np.uint16), npre)
    rn = np.where(rng.random(npre) < 0.6, raw16(rng.integers(1, 11, npre)), 0).astype(np.uint16)
    rv = ct_vals(npre, 4000, 0, 0, 300, rx=(2, 200))
    rv[:, 36:38] = le_bytes(fl, "<u2")
    rv[:, 38:40] = le_bytes(rn, "<u2")
    k, v = dedup(np.concatenate([ct.keys, rk, relk, estk]),
                 np.concatenate([ct.vals, rv, rv, ct_vals(npre, 4000, 16, 0, 256 + np.arange(npre) % 4)]))
    ct.keys, ct.vals = k, v
    pool = dict(e=rng.integers(0, n_ep, npre), d=R, sp=a, dp=b, pr=pr)
    pool["e"] = np.searchsorted(ep4, E)
    # ---- packets
    for bi in range(n_batches):
        n = n_packets
        kind = rng.random(n)
        e = rng.integers(0, n_ep, n)
        peer = rng.integers(0, n_ep, n) if hazard else (e + 1 + rng.integers(0, n_ep - 1, n)) % n_ep
        lo = np.uint32(ip4("10.255.255.245")) if hazard else rem4[3]
        d = np.where(kind < 0.30, vip4[rng.integers(0, 8, n)],
                     np.where(kind < 0.55, ep4[peer],
                              np.where(kind < 0.85, rem4[rng.integers(0, len(rem4), n)],
                                       np.where(kind < 0.90, lo,
                                                rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)))))
        pr = rng.choice(np.array([TCP, TCP, TCP, UDP, UDP, ICMP, ICMP, 47], np.uint8), n)
        sp = np.where(rng.random(n) < 0.3, 30000 + rng.integers(0, 20, n), ports[rng.integers(0, len(ports), n)])
        dp = ports[rng.integers(0, len(ports), n)]
        use = rng.random(n) < 0.35                     # the pre-populated flows, both directions
        pi = rng.integers(0, npre, n)
        e = np.where(use, pool["e"][pi], e)
        d = np.where(use, pool["d"][pi], d)
        pr = np.where(use, pool["pr"][pi], pr).astype(np.uint8)
        if not icmp:                                   # no IPv4 ICMP: the connection-group schedule holds
            pr = np.where(pr == ICMP, UDP, pr).astype(np.uint8)
        sp = np.where(use, pool["sp"][pi], sp)
        dp = np.where(use, pool["dp"][pi], dp)
        s = ep4[e].copy()
        bad_sip = rng.random(n) < 0.02
        s[bad_sip] = rem4[rng.integers(0, len(rem4), int(bad_sip.sum()))]
        tf = rng.choice(np.array([F_SYN, F_ACK, F_ACK, F_FIN | F_ACK, F_RST, F_SYN | F_ACK], np.uint8), n)
        it = rng.choice(np.array([0, 3, 8, 8, 11, 12, 5], np.uint8), n)
        ihl = np.where(rng.random(n) < 0.05, rng.integers(0, 16, n), 5)
        f, lens = frames_v4(n, 256, s, d, pr, sp, dp, tf, it, 0, ihl, payload=rng.integers(0, 64, n))
        f[:, 6:12] = macs[e]
        f[rng.random(n) < 0.02, 6] ^= 1
        f[:, 0:6] = np.frombuffer(node_mac, np.uint8)
        f[rng.random(n) < 0.02, 0] ^= 1
        ttl = np.where(rng.random(n) < 0.05, rng.integers(0, 2, n), rng.integers(2, 256, n)).astype(np.uint8)
        f[:, 22] = ttl
        f[:, 24:26] = rng.integers(0, 256, (n, 2))
        l4 = 14 + (f[:, 14] & 0xf).astype(np.int64) * 4
        off = np.where(pr == 6, l4 + 16, np.where(pr == 17, l4 + 6, -1))
        ck = rng.integers(0, 65536, n)
        ck[rng.random(n) < 0.1] = 0
        ok = (off >= 0) & (off + 1 < f.shape[1])
        rows = np.nonzero(ok)[0]
        f[rows, off[ok]] = (ck[ok] >> 8).astype(np.uint8)
        f[rows, off[ok] + 1] = (ck[ok] & 0xff).astype(np.uint8)
        oth = rng.random(n)
        i6 = np.nonzero(oth < 0.18)[0]                 # IPv6 from the endpoints (ipv6_l3_from_lxc)
        m = len(i6)
        if m:
            e6 = e[i6]
            k6 = rng.random(m)
            peer6 = ep6[(e6 + 1 + rng.integers(0, n_ep - 1, m)) % n_ep] if not hazard else ep6[rng.integers(0, n_ep, m)]
            rtr = np.frombuffer(router6, np.uint8)
            clus = np.tile(rtr, (m, 1)); clus[:, 8:] = rng.integers(0, 256, (m, 8))
            tun6 = np.tile(rem6[7], (m, 1)); tun6[:, 12:] = rng.integers(0, 256, (m, 4))
            d6 = np.where((k6 < 0.25)[:, None], vip6[rng.integers(0, len(vip6), m)],
                          np.where((k6 < 0.45)[:, None], peer6,
                                   np.where((k6 < 0.75)[:, None], rem6[rng.integers(0, len(rem6), m)],
                                            np.where((k6 < 0.85)[:, None], clus,
                                                     np.where((k6 < 0.92)[:, None], tun6, np.tile(rtr, (m, 1)))))))
            s6 = ep6[e6].copy()
            bad6 = rng.random(m) < 0.03
            s6[bad6] = rem6[rng.integers(0, len(rem6), int(bad6.sum()))]
            nh6 = rng.choice(np.array([TCP, TCP, UDP, ICMPV6, ICMPV6, 47], np.uint8), m)
            it6 = rng.choice(np.array([128, 129, 135, 1, 3, 2, 136], np.uint8), m)
            ext = []
            depth = np.where(rng.random(m) < 0.15, rng.integers(1, 6, m), 0)
            for lvl in range(5):
                t = rng.choice(np.array([0, 60, 43, 51, 44, 59, 0], np.uint8), m)
                ext.append((np.where(depth > lvl, t, 255).astype(np.uint8), rng.integers(0, 3, m).astype(np.uint8)))
            f6, l6 = frames_v6(m, 256, s6, d6, nh6, sp[i6], dp[i6], tf[i6], it6, ext=ext, payload=rng.integers(0, 64, m))
            f6[:, 6:12] = macs[e6]
            f6[:, 0:6] = np.frombuffer(node_mac, np.uint8)
            f6[rng.random(m) < 0.02, 6] ^= 1
            f6[:, 21] = np.where(rng.random(m) < 0.05, rng.integers(0, 2, m), rng.integers(2, 256, m))
            ok6 = (nh6 == 6) | (nh6 == 17)
            f[i6] = f6
            lens[i6] = l6
        ia = np.nonzero((oth >= 0.18) & (oth < 0.20))[0]
        f[ia, 12], f[ia, 13] = 0x08, 0x06
        io = np.nonzero((oth >= 0.20) & (oth < 0.21))[0]
        f[io, 12], f[io, 13] = 0x88, 0xcc
        lens = lens.astype(np.int64)
        tr = rng.random(n) < 0.06
        lens[tr] = rng.integers(0, np.maximum(lens[tr], 1) + 1)
        lens = np.minimum(lens, 256 + 400).astype(np.uint32)
        lid = np.where(rng.random(n) < 0.98, lxc_id[e], 4242).astype(np.uint16)
        fh = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        sc.batches.append(Packets(f, lens, None, None, lid, None, fh))
    return sc


TENANT = 256     # endpoints per tenant in the egress workload (256: one tenant, every endpoint talks to every other)


def egress_tables(n_ep=256, n_svc=1024, backends=4, ct_max=64_000_000, seed=0xE6E5):
    """Egress measurement tables (the agent's production flag set: no
    POLICY_EGRESS): n_ep local endpoints (10.1.x.y) with their MACs, one global
    CT map, services whose backends are local endpoints (so some translate back
    to the sender: loopback SNAT), a tunnel map covering 10.128.0.0/16, and
    per-endpoint ingress policy admitting the endpoints' identities (local
    deliveries continue into handle_policy).  Endpoints form tenants of TENANT
    (endpoint e is in tenant e // TENANT); service s belongs to tenant
    s % (n_ep // TENANT) and its backends are that tenant's endpoints, so local
    traffic never crosses tenants and a tenant is a closed set of flow groups
    (the bench's parity sample)."""
    rng = np.random.default_rng(seed)
    sc = Scenario("egress_bench", now=10_000, host_ifindex=3)
    ep4 = (ip4("10.1.0.0") + 1 + np.arange(n_ep)).astype(np.uint32)
    lxc_id = (1000 + np.arange(n_ep)).astype(np.uint32)
    seclabel = (256 + np.arange(n_ep)).astype(np.uint32)
    macs = rng.integers(0, 256, (n_ep, 6)).astype(np.uint8)
    node_mac = bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])
    ev = endpoint_infos(10 + np.arange(n_ep), seclabel, lxc_id, np.zeros(n_ep))
    ev[:, 16:22] = macs
    ev[:, 24:30] = np.frombuffer(node_mac, np.uint8)
    sc.add_map(MapSpec("cilium_lxc", HASH, 20, 112, 65535, 0, endpoint_keys4(ep4), ev))
    sc.add_map(MapSpec("ct4", LRU_HASH, 14, 48, ct_max, 0))
    sc.add_map(MapSpec("ct6", LRU_HASH, 40, 48, 1 << 16, 0))
    vip = (ip4("10.96.0.0") + 1 + np.arange(n_svc)).astype(np.uint32)
    sport = rng.choice(np.array([80, 443, 8080, 53], np.uint32), n_svc)
    nten = n_ep // TENANT
    tgt = ep4[(np.arange(n_svc) % nten)[:, None] * TENANT + rng.integers(0, TENANT, (n_svc, backends))]
    keys = [lb4_keys(vip, sport, np.zeros(n_svc))]
    vals = [lb4_vals(np.zeros(n_svc), np.zeros(n_svc), np.full(n_svc, backends), np.zeros(n_svc))]
    for b in range(backends):
        keys.append(lb4_keys(vip, sport, np.full(n_svc, b + 1)))
        vals.append(lb4_vals(tgt[:, b], np.where(np.arange(n_svc) % 3 == 0, 8080, sport), np.zeros(n_svc),
                             1 + np.arange(n_svc)))
    sc.add_map(MapSpec("lb4", HASH, 8, 12, 1 << 20, 0, np.concatenate(keys), np.concatenate(vals)))
    rk, rv = revnat4_entries(1 + np.arange(n_svc), vip, sport)
    sc.add_map(MapSpec("revnat4", HASH, 2, 6, 1 << 16, 0, rk, rv))
    sc.add_map(MapSpec("tunnel", HASH, 20, 20, 65536, 0, endpoint_keys4(np.array([ip4("10.128.0.0")], np.uint32)),
                       endpoint_keys4(np.array([ip4("192.168.7.2")], np.uint32))))
    pk = policy_keys(seclabel, np.zeros(n_ep), np.zeros(n_ep))
    pv = policy_vals(np.zeros(n_ep))
    for e in range(n_ep):
        sc.add_map(MapSpec(f"pol{e}", HASH, 8, 24, 16384, 0, pk, pv))
        sc.lxc.append({"lxc_id": int(lxc_id[e]), "seclabel": int(seclabel[e]), "policy": f"pol{e}", "ct4": "ct4",
                       "ct6": "ct6", "revnat4": "revnat4", "flags": LXC_PRODUCTION, "lxc_mac": bytes(macs[e]),
                       "node_mac": node_mac, "lxc_ipv4": int(be32_bytes([ep4[e]]).view("<u4")[0, 0]), "lb4": "lb4"})
    raw_be = lambda a: int(be32_bytes([a]).view("<u4")[0, 0])
    sc.node = {"lxc_map": "cilium_lxc", "ipv4_cluster_range": raw_be(ip4("10.0.0.0")),
               "ipv4_cluster_mask": raw_be(0xFF000000), "ipv4_loopback": raw_be(ip4("10.255.255.245")),
               "ipv4_mask": raw_be(0xFFFF0000), "encap_ifindex": 5, "tunnel_map": "tunnel",
               "host_mac": bytes([0xce, 0x72, 0xa7, 0x03, 0x88, 0x56]), "node_mac": node_mac}
    meta = dict(ep4=ep4, lxc_id=lxc_id, macs=macs, vip=vip, sport=sport, node_mac=node_mac)
    return sc, meta


def egress_flows(meta, n_flows, seed=0xE6E6):
    """n_flows egress flows (one frame each, 64-B snaps): 35% world peers (to the
    stack), 20% tunnel peers (encap), 25% other local endpoints (local delivery),
    20% service VIPs (lb4_local to a local backend).  Returns (frames, lens,
    lxc_id, flow_hash, sport column offset)."""
    rng = np.random.default_rng(seed)
    ep4, n_ep = meta["ep4"], len(meta["ep4"])
    e = rng.integers(0, n_ep, n_flows)
    kind = rng.random(n_flows)
    world = (ip4("100.64.0.0") + rng.integers(0, 1 << 20, n_flows)).astype(np.uint32)
    tun = (ip4("10.128.0.0") + rng.integers(0, 1 << 16, n_flows)).astype(np.uint32)
    ten, nten = e // TENANT, n_ep // TENANT                # local peers and services of the own tenant
    peer = ep4[ten * TENANT + (e % TENANT + 1 + rng.integers(0, TENANT - 1, n_flows)) % TENANT]
    si = ten + nten * rng.integers(0, len(meta["vip"]) // nten, n_flows)
    d = np.where(kind < 0.35, world, np.where(kind < 0.55, tun, np.where(kind < 0.80, peer, meta["vip"][si])))
    dp = np.where(kind >= 0.80, meta["sport"][si], rng.choice(np.array([80, 443, 53, 8080], np.uint32), n_flows))
    pr = np.where(rng.random(n_flows) < 0.8, TCP, UDP).astype(np.uint8)
    sp = 1024 + rng.integers(0, 60000, n_flows)
    f, lens = frames_v4(n_flows, 64, ep4[e], d, pr, sp, dp, F_ACK, payload=rng.integers(0, 64, n_flows))
    f[:, 6:12] = meta["macs"][e]
    f[:, 0:6] = np.frombuffer(meta["node_mac"], np.uint8)
    fh = rng.integers(0, 1 << 32, n_flows, dtype=np.uint64).astype(np.uint32)
    return f, lens, meta["lxc_id"][e].astype(np.uint16), fh
