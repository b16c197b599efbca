"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (see oracle.h)."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "liboracle.so")
if not os.path.exists(_PATH):
    raise ImportError(f"{_PATH} missing: run `make -C oracle`")
lib = C.CDLL(_PATH)
VP = C.c_void_p


class o_l4_allow(C.Structure):
    _fields_ = [("port", C.c_uint16), ("proxy", C.c_uint16), ("nexthdr", C.c_uint8), ("pad", C.c_uint8 * 3)]


class o_xdp_cfg(C.Structure):
    _fields_ = [("cidr4_hmap", VP), ("cidr4_lmap", VP), ("cidr6_hmap", VP), ("cidr6_lmap", VP), ("lxc_map", VP)]


class o_lb_cfg(C.Structure):
    _fields_ = [("lb4_services", VP), ("lb6_services", VP), ("flags", C.c_uint32), ("redirect_ifindex", C.c_uint32)]


class o_lxc_cfg(C.Structure):
    _fields_ = [("lxc_id", C.c_uint32), ("seclabel", C.c_uint32), ("policy_map", VP), ("ct_map4", VP),
                ("ct_map6", VP), ("cidr4_ingress_map", VP), ("cidr6_ingress_map", VP), ("revnat4_map", VP),
                ("revnat6_map", VP), ("flags", C.c_uint32), ("n_l4_ingress", C.c_uint32),
                ("l4_ingress", o_l4_allow * 64), ("lxc_mac", C.c_uint8 * 6), ("node_mac", C.c_uint8 * 6),
                ("lxc_ipv4", C.c_uint32), ("lb4_services", VP), ("ipcache_map", VP), ("cidr4_egress_map", VP),
                ("n_portmap", C.c_uint32), ("portmap", C.c_uint16 * 32), ("n_l4_egress", C.c_uint32),
                ("l4_egress", o_l4_allow * 64), ("lxc_ip6", C.c_uint8 * 16), ("lb6_services", VP),
                ("cidr6_egress_map", VP)]


class o_node_cfg(C.Structure):
    _fields_ = [("host_ifindex", C.c_uint32), ("proxy4_map", VP), ("proxy6_map", VP), ("ipv4_gateway", C.c_uint32),
                ("host_ip6", C.c_uint8 * 16), ("host_mac", C.c_uint8 * 6), ("node_mac", C.c_uint8 * 6),
                ("lxc_map", VP), ("ipv4_cluster_range", C.c_uint32), ("ipv4_cluster_mask", C.c_uint32),
                ("ipv4_loopback", C.c_uint32), ("ipv4_mask", C.c_uint32), ("encap_ifindex", C.c_uint32),
                ("tunnel_map", VP), ("router_ip6", C.c_uint8 * 16)]


class o_batch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("snap_stride", C.c_uint32), ("snap", VP), ("len", VP),
                ("src_identity", VP), ("ifindex", VP), ("flow_hash", VP), ("lxc_id", VP), ("tc_index", VP)]


class o_cols(C.Structure):
    _fields_ = [("ethertype", VP), ("saddr4", VP), ("daddr4", VP), ("proto", VP), ("l4_off", VP),
                ("l4w0", VP), ("l4w3", VP), ("saddr6", VP), ("daddr6", VP)]


class o_netdev_cfg(C.Structure):
    _fields_ = [("lxc_map", VP), ("flags", C.c_uint32), ("fixed_secctx", C.c_uint32), ("router_ip6", C.c_uint8 * 16),
                ("ingress_ifindex", C.c_uint32)]


class o_pipeline_cfg(C.Structure):
    _fields_ = [("xdp", C.POINTER(o_xdp_cfg)), ("lb", C.POINTER(o_lb_cfg)), ("netdev", C.POINTER(o_netdev_cfg)),
                ("policy", VP)]


def _s(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)


_s("om_create", VP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32)
_s("om_destroy", None, VP)
_s("om_update", C.c_int, VP, VP, VP, C.c_uint64)
_s("om_lookup", C.c_int, VP, VP, VP)
_s("om_delete", C.c_int, VP, VP)
_s("om_update_many", C.c_int, VP, VP, VP, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint32))
_s("om_count", C.c_uint32, VP)
_s("om_dump", C.c_uint32, VP, VP, VP, C.c_uint32)
_s("o_parse_batch", None, C.POINTER(o_batch), C.POINTER(o_cols))
_s("o_xdp_batch", None, C.POINTER(o_xdp_cfg), C.POINTER(o_batch), VP)
_s("o_xdp_batch_mt", None, C.POINTER(o_xdp_cfg), C.POINTER(o_batch), VP, C.c_uint32)
_s("o_lb_batch", None, C.POINTER(o_lb_cfg), C.POINTER(o_batch), VP, VP)
_s("o_lb_batch_mt", None, C.POINTER(o_lb_cfg), C.POINTER(o_batch), VP, VP, C.c_uint32)
_s("o_prog_array_create", VP)
_s("o_prog_array_destroy", None, VP)
_s("o_prog_array_set", None, VP, C.c_uint32, C.POINTER(o_lxc_cfg))
_s("o_set_node", None, C.POINTER(o_node_cfg))
_s("o_ingress_batch", None, VP, C.POINTER(o_batch), C.c_uint32, VP)
_s("o_ingress_batch_mt", None, VP, C.POINTER(o_batch), C.c_uint32, VP, C.c_uint32)
_s("o_pipeline_batch_mt", None, C.POINTER(o_pipeline_cfg), C.POINTER(o_batch), C.c_uint32, VP, VP, VP, C.c_uint32, VP)
_s("o_ingress_events", None, VP, C.POINTER(o_batch), VP, VP)
_s("o_set_trace_sink", None, VP, VP, C.c_uint32, C.c_int)
_s("o_egress_batch", None, VP, C.POINTER(o_batch), C.c_uint32, VP, VP, VP)
_s("o_ct_gc", C.c_uint32, VP, C.c_uint32)
_s("o_ct_lru_evict", C.c_int, VP, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
   C.POINTER(C.c_uint64))
_s("o_ct_lru_replay", C.c_uint64, VP, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64)
_s("o_rows_fp", None, VP, VP, C.c_uint64, C.c_uint32, C.c_uint32, VP)
_s("o_get_prefix", C.c_uint32, C.c_int)
_s("o_ipv6_addr_clear_suffix", None, VP, C.c_int)
_s("o_lpm4_iter_lookup", C.c_int, C.c_uint32, VP, C.c_int, C.c_uint32)
_s("o_ct_pair_hash4", C.c_uint32, C.c_uint32, C.c_uint32)

def rows_fp(keys, vals):
    """64-bit fingerprints of the (key, value) rows of a dump (uint64[n])."""
    k = np.ascontiguousarray(keys, np.uint8)
    v = np.ascontiguousarray(vals, np.uint8)
    out = np.empty(len(k), np.uint64)
    n, ks, vs = len(k), k.shape[1] if k.ndim == 2 else 0, v.shape[1] if v.ndim == 2 else 0
    if not n:
        return out
    nt = min(16, os.cpu_count() or 1, max(1, n // (1 << 20)))
    step = (n + nt - 1) // nt

    def part(a):                      # ctypes drops the GIL: the chunks run in parallel
        b = min(n, a + step)
        lib.o_rows_fp(k.ctypes.data + a * ks, v.ctypes.data + a * vs, b - a, ks, vs, out.ctypes.data + 8 * a)
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(nt) as ex:
        list(ex.map(part, range(0, n, step)))
    return out


LB_OUT = np.dtype([("action", "u1"), ("reason", "u1"), ("slave", "<u2"), ("new_dport", "<u2"),
                   ("rev_nat", "<u2"), ("new_daddr4", "<u4")])
ING_OUT = np.dtype([("action", "u1"), ("reason", "u1"), ("ct_ret", "u1"), ("flags", "u1"),
                    ("proxy_port", "<u2"), ("ifindex_lo", "<u2")])
PIPE_OUT = np.dtype([("stage", "u1"), ("action", "u1"), ("reason", "u1"), ("ct_ret", "u1"), ("flags", "u1"),
                     ("pad0", "u1"), ("proxy_port", "<u2"), ("ifindex_lo", "<u2"), ("slave", "<u2"),
                     ("rev_nat", "<u2"), ("dport", "<u2"), ("daddr4", "<u4"), ("lxc_id", "<u2"), ("pad1", "<u2")])
EG_OUT = np.dtype([("stage", "u1"), ("action", "u1"), ("reason", "u1"), ("ct_ret", "u1"), ("flags", "u1"),
                   ("eg_ct_ret", "u1"), ("proxy_port", "<u2"), ("ifindex_lo", "<u2"), ("slave", "<u2"),
                   ("rev_nat", "<u2"), ("eg_flags", "<u2"), ("tunnel_ip", "<u4"), ("lxc_id", "<u2"), ("pad", "<u2")])


class OMap:
    """One oracle map (kernel htab / LPM trie semantics)."""

    def __init__(self, typ, ksz, vsz, max_entries, shards=1):
        self.ptr = lib.om_create(typ, ksz, vsz, max_entries, shards)
        if not self.ptr:
            raise ValueError("om_create failed")
        self.ksz, self.vsz = ksz, vsz

    def update(self, key, value, flags=0):
        return lib.om_update(self.ptr, key, value, flags)

    def update_many(self, keys, values, flags=0):
        k = np.ascontiguousarray(keys, np.uint8).reshape(-1)
        v = np.ascontiguousarray(values, np.uint8).reshape(-1)
        n = len(k) // self.ksz
        done = C.c_uint32(0)
        rc = lib.om_update_many(self.ptr, k.ctypes.data, v.ctypes.data, n, flags, C.byref(done))
        if rc:
            raise OSError(-rc, f"om_update (entry {done.value})")

    def lookup(self, key):
        v = C.create_string_buffer(self.vsz)
        rc = lib.om_lookup(self.ptr, key, v)
        return None if rc else v.raw

    def delete(self, key):
        return lib.om_delete(self.ptr, key)

    def count(self):
        return lib.om_count(self.ptr)

    def ct_gc(self, filter_time):
        return lib.o_ct_gc(self.ptr, filter_time)

    def lru_evict(self, now):
        """The LRU stand-in after a batch on this map's own contents: None (no
        eviction) or the log record (age_cut, hand_line, lines, evicted)."""
        k, h, ln, ev = C.c_uint32(0), C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        if not lib.o_ct_lru_evict(self.ptr, now, C.byref(k), C.byref(h), C.byref(ln), C.byref(ev)):
            return None
        return k.value, h.value, ln.value, ev.value

    def lru_replay(self, now, age_cut, hand, lines):
        """A logged eviction replayed; returns the entries deleted."""
        return lib.o_ct_lru_replay(self.ptr, now, age_cut, hand, lines)

    def dump_arrays(self):
        """All entries as (keys uint8[n, ksz], values uint8[n, vsz])."""
        n = self.count()
        k = np.zeros((max(1, n), self.ksz), np.uint8)
        v = np.zeros((max(1, n), self.vsz), np.uint8)
        m = lib.om_dump(self.ptr, k.ctypes.data, v.ctypes.data, n)
        return k[:min(m, n)], v[:min(m, n)]

    def dump(self):
        n = self.count()
        kb = C.create_string_buffer(max(1, n * self.ksz))
        vb = C.create_string_buffer(max(1, n * self.vsz))
        m = lib.om_dump(self.ptr, kb, vb, n)
        return {kb.raw[i * self.ksz:(i + 1) * self.ksz]: vb.raw[i * self.vsz:(i + 1) * self.vsz] for i in range(m)}

    def __del__(self):
        try:
            if self.ptr:
                lib.om_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass


def make_batch(frames, lens, src_identity=None, ifindex=None, lxc_id=None, tc_index=None, flow_hash=None):
    """Builds an o_batch over numpy arrays (kept alive on the returned object)."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    keep = [frames]
    b = o_batch()
    b.n = frames.shape[0]
    b.snap_stride = frames.shape[1]
    b.snap = frames.ctypes.data

    def arr(x, dt):
        if x is None:
            return None
        a = np.ascontiguousarray(x, dtype=dt)
        keep.append(a)
        return a.ctypes.data

    b.len = arr(lens, np.uint32)
    b.src_identity = arr(src_identity, np.uint32)
    b.ifindex = arr(ifindex, np.uint32)
    b.lxc_id = arr(lxc_id, np.uint16)
    b.tc_index = arr(tc_index, np.uint8)
    b.flow_hash = arr(flow_hash, np.uint32)
    b._keep = keep
    return b


def parse(b):
    n = b.n
    out = {"ethertype": np.zeros(n, np.uint16), "saddr4": np.zeros(n, np.uint32), "daddr4": np.zeros(n, np.uint32),
           "proto": np.zeros(n, np.uint8), "l4_off": np.zeros(n, np.int16), "l4w0": np.zeros(n, np.uint32),
           "l4w3": np.zeros(n, np.uint16), "saddr6": np.zeros((n, 16), np.uint8), "daddr6": np.zeros((n, 16), np.uint8)}
    c = o_cols(*[out[k].ctypes.data for k in ("ethertype", "saddr4", "daddr4", "proto", "l4_off", "l4w0", "l4w3",
                                               "saddr6", "daddr6")])
    lib.o_parse_batch(C.byref(b), C.byref(c))
    return out


def xdp(cfg, b, threads=1):
    v = np.zeros(b.n, np.uint8)
    if threads > 1:
        lib.o_xdp_batch_mt(C.byref(cfg), C.byref(b), v.ctypes.data, threads)
    else:
        lib.o_xdp_batch(C.byref(cfg), C.byref(b), v.ctypes.data)
    return v


def lb(cfg, b, threads=1):
    out = np.zeros(b.n, LB_OUT)
    nd6 = np.zeros((b.n, 16), np.uint8)
    if threads > 1:
        lib.o_lb_batch_mt(C.byref(cfg), C.byref(b), out.ctypes.data, nd6.ctypes.data, threads)
    else:
        lib.o_lb_batch(C.byref(cfg), C.byref(b), out.ctypes.data, nd6.ctypes.data)
    return out, nd6


def ingress(prog_array, b, now, threads=1):
    out = np.zeros(b.n, ING_OUT)
    if threads > 1:
        lib.o_ingress_batch_mt(prog_array, C.byref(b), now, out.ctypes.data, threads)
    else:
        lib.o_ingress_batch(prog_array, C.byref(b), now, out.ctypes.data)
    return out


def pipeline(cfg, b, now, threads=1, events=False):
    """o_pipeline_batch_mt: returns (records, new_daddr6, rewritten snaps[, drop events in batch order])."""
    out = np.zeros(b.n, PIPE_OUT)
    nd6 = np.zeros((b.n, 16), np.uint8)
    snap = np.zeros((b.n, b.snap_stride), np.uint8)
    ev = np.zeros((b.n, 160), np.uint8) if events else None
    lib.o_pipeline_batch_mt(C.byref(cfg), C.byref(b), now, out.ctypes.data, nd6.ctypes.data, snap.ctypes.data,
                            max(1, threads), None if ev is None else ev.ctypes.data)
    if events:
        return out, nd6, snap, ev[ev[:, 0] == 1]
    return out, nd6, snap


class TraceSink:
    """o_set_trace_sink for the calls inside a `with` block: each packet's trace
    records (trace.h:59-106) then its drop record, per packet in emission order.
    .events() = every record in batch order ([k, 160] u8), the ring's order."""
    PER = 4

    def __init__(self, n, capture=True):
        self.ev = np.zeros((n, self.PER, 160), np.uint8)
        self.cnt = np.zeros(n, np.uint8)
        self.capture = capture

    def __enter__(self):
        lib.o_set_trace_sink(self.ev.ctypes.data, self.cnt.ctypes.data, self.PER, 1 if self.capture else 0)
        return self

    def __exit__(self, *a):
        lib.o_set_trace_sink(None, None, 0, 0)

    def events(self):
        k = np.arange(self.PER)[None, :] < self.cnt[:, None]
        return self.ev[k]


def ingress_events(prog_array, b, out):
    """Drop notifications of an ingress batch, in batch order ([k, 160] u8)."""
    ev = np.zeros((b.n, 160), np.uint8)
    lib.o_ingress_events(prog_array, C.byref(b), out.ctypes.data, ev.ctypes.data)
    return ev[ev[:, 0] == 1]


def egress(prog_array, b, now, events=False):
    """o_egress_batch: returns (records EG_OUT, rewritten snaps[, drop events in batch order])."""
    out = np.zeros(b.n, EG_OUT)
    snap = np.zeros((b.n, b.snap_stride), np.uint8)
    ev = np.zeros((b.n, 160), np.uint8) if events else None
    lib.o_egress_batch(prog_array, C.byref(b), now, out.ctypes.data, snap.ctypes.data,
                       None if ev is None else ev.ctypes.data)
    if events:
        return out, snap, ev[ev[:, 0] == 1]
    return out, snap
