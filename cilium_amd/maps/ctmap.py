"""pkg/maps/ctmap mirror (/root/reference/pkg/maps/ctmap/{ctmap,ipv4,ipv6}.go).

CtKey4Global = struct ipv4_ct_tuple (14 B, packed): daddr, saddr, dport(be), sport(be), nexthdr, flags
CtKey6Global = struct ipv6_ct_tuple (40 B)
CtEntry (48 B): rx_packets, rx_bytes, tx_packets, tx_bytes, lifetime u32, flags u16,
                revnat u16 (network order), unused u16, pad u16, src_sec_id u32
GC (ctmap.go:277-352) deletes entries whose lifetime < now; Flush (:354-368)
deletes every entry.  Both go to gf_ct_gc: a device sweep of the HBM replica
(with probe-cluster compaction) when the datapath owns the map.
"""
import errno
import struct

from .. import bpf

MapName6, MapName4 = "cilium_ct6_", "cilium_ct4_"
MapName6Global, MapName4Global = MapName6 + "global", MapName4 + "global"
MapNumEntriesLocal, MapNumEntriesGlobal = 64000, 1000000
TUPLE_F_OUT, TUPLE_F_IN, TUPLE_F_RELATED = 0, 1, 2
KEY4 = struct.Struct("<IIHHBB")
KEY6 = struct.Struct("<16s16sHHBB2s")
ENTRY = struct.Struct("<QQQQIHHHHI")


def MapNames(ep_id=None, local=False):
    """The CT maps an endpoint's program binds (pkg/endpoint/bpf.go:268-276): with the
    ConntrackLocal option its own cilium_ct6_<id> / cilium_ct4_<id> of CT_MAP_SIZE
    MapNumEntriesLocal, else the global ones of MapNumEntriesGlobal.  Returns
    (CT_MAP6 name, CT_MAP4 name, CT_MAP_SIZE); the classify calls take either kind, mixed
    in one program array (include/gpuflow.h, gf_lxc_cfg.ct_map4)."""
    if local:
        if ep_id is None:
            raise ValueError("a per-endpoint CT map needs the endpoint ID")
        return MapName6 + str(int(ep_id)), MapName4 + str(int(ep_id)), MapNumEntriesLocal
    return MapName6Global, MapName4Global, MapNumEntriesGlobal


def ct_key4(daddr_be, saddr_be, dport_be, sport_be, nexthdr, flags):
    return KEY4.pack(daddr_be, saddr_be, dport_be, sport_be, nexthdr, flags)


def ct_key6(daddr, saddr, dport_be, sport_be, nexthdr, flags):
    return KEY6.pack(daddr, saddr, dport_be, sport_be, nexthdr, flags, b"\x00\x00")


def ct_entry(rx_packets=0, rx_bytes=0, tx_packets=0, tx_bytes=0, lifetime=0, flags=0,
             revnat=0, src_sec_id=0):
    return ENTRY.pack(rx_packets, rx_bytes, tx_packets, tx_bytes, lifetime, flags, revnat, 0, 0, src_sec_id)


class CtEntry:
    def __init__(self, raw):
        (self.rx_packets, self.rx_bytes, self.tx_packets, self.tx_bytes, self.lifetime, self.flags,
         self.revnat, self.unused, _, self.src_sec_id) = ENTRY.unpack(raw)


def OpenMap(path, v6=False, max_entries=MapNumEntriesGlobal, lru=True):
    typ = bpf.BPF_MAP_TYPE_LRU_HASH if lru else bpf.BPF_MAP_TYPE_HASH
    ks = KEY6.size if v6 else KEY4.size
    fd, new = bpf.OpenOrCreateMap(path, typ, ks, ENTRY.size, max_entries, 0)
    return fd, new


def Dump(fd, v6=False):
    ks = KEY6.size if v6 else KEY4.size
    out = []
    key = None
    while True:
        try:
            nk = bpf.GetNextKey(fd, key, ks)
        except bpf.BPFError as e:
            if e.errno == errno.ENOENT:
                return out
            raise
        out.append((nk, CtEntry(bpf.LookupElement(fd, nk, ENTRY.size))))
        key = nk


MaxTime = 0xFFFFFFFF


def GC(fd, now_sec, v6=False):
    """doGC4/doGC6 + doFiltering (GCFilterByTime): delete lifetime < now; returns
    the number of entries deleted."""
    from .._lib import lib
    rc = lib.gf_ct_gc(fd, now_sec & 0xFFFFFFFF, None)
    if rc < 0:
        raise bpf.BPFError(-rc, "Unable to garbage collect CT map")
    return rc


def Flush(fd, v6=False):
    """ctmap.Flush: GC with filter time MaxTime (every entry)."""
    return GC(fd, MaxTime, v6)
