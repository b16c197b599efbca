"""Host side of the datapath: load programs over maps and run classify calls.

This mirrors what the agent does in the reference: create/pin maps through
pkg/bpf (here cilium_amd.bpf over libgpuflow), generate the per-endpoint
configuration (pkg/endpoint/bpf.go:156-330 -> gf_lxc_cfg instead of a
compiled header), install the tail-call slots (cilium_policy prog array) and
then let packets flow — here, batches resident in HBM.

Batches are torch tensors on the current CUDA/HIP device; PyTorch is only the
allocator/stream provider, every computation runs in libgpuflow's kernels.
"""
import ctypes as C
import errno

import numpy as np

from . import bpf
from ._lib import (lib, gf_frames, gf_pkt_cols, gf_pkt_cols_out, gf_xdp_cfg, gf_lb_cfg, gf_lxc_cfg,
                   gf_node_cfg, gf_netdev_cfg, gf_pipeline_cfg, gf_pipe_batch, gf_lxc_batch)

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


def _be16(x):
    return ((x & 0xff) << 8) | (x >> 8)


def egress_fields(c, e, h):
    """The from-container section of an endpoint's gf_lxc_cfg (pkg/endpoint/bpf.go:156-330
    emits these as LXC_MAC, NODE_MAC, LXC_IPV4, LXC_PORT_MAPPINGS, CFG_L3L4_EGRESS)."""
    c.lxc_mac[:] = list(e.get("lxc_mac", bytes(6)))
    c.node_mac[:] = list(e.get("node_mac", bytes(6)))
    c.lxc_ipv4 = e.get("lxc_ipv4", 0)
    c.lb4_services, c.ipcache_map, c.cidr4_egress_map = h(e.get("lb4")), h(e.get("ipcache")), h(e.get("cidr4e"))
    c.lb6_services, c.cidr6_egress_map = h(e.get("lb6")), h(e.get("cidr6e"))
    c.lxc_ip6[:] = list(e.get("lxc_ip6", bytes(16)))
    pm = e.get("portmap") or []
    c.n_portmap = len(pm)
    for i, (frm, to) in enumerate(pm):
        c.portmap[2 * i], c.portmap[2 * i + 1] = _be16(frm), _be16(to)
    l4 = e.get("l4e") or []
    c.n_l4_egress = len(l4)
    for i, (port, proxy, nh) in enumerate(l4):
        c.l4_egress[i].port, c.l4_egress[i].proxy, c.l4_egress[i].nexthdr = _be16(port), _be16(proxy), nh


def _torch():
    import torch
    return torch


def _check(rc, what):
    if rc < 0:
        raise OSError(-rc, f"{what}: {errno.errorcode.get(-rc, rc)}")
    return rc


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream():
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class DeviceBatch:
    """Raw frames + skb metadata uploaded to HBM, parsed into SoA columns by
    gf_parse_frames (k_parse)."""

    def __init__(self, pk, device="cuda", parse=True, with_v6=True):
        torch = _torch()
        self.n = pk.n
        self.device = device
        signed = {np.dtype(np.uint32): np.int32, np.dtype(np.uint16): np.int16, np.dtype(np.uint8): np.uint8}

        def t(a, dt):
            if a is None:
                return None
            a = np.ascontiguousarray(np.asarray(a).astype(dt, copy=False))
            return torch.from_numpy(a.view(signed[np.dtype(dt)])).to(device)

        self.frames = t(pk.frames, np.uint8)
        self.len = t(pk.lens, np.uint32)
        self.src_identity = t(pk.src_identity, np.uint32)
        self.ifindex = t(pk.ifindex, np.uint32)
        self.lxc_id = t(pk.lxc_id, np.uint16)
        self.tc_index = t(pk.tc_index, np.uint8)
        self.flow_hash = t(pk.flow_hash, np.uint32)
        n = self.n
        e = lambda dt, *shape: torch.empty((n,) + shape, dtype=dt, device=device)
        self.ethertype = e(torch.int16)
        self.saddr4 = e(torch.int32)
        self.daddr4 = e(torch.int32)
        self.proto = e(torch.uint8)
        self.l4_off = e(torch.int16)
        self.l4w0 = e(torch.int32)
        self.l4w3 = e(torch.int16)
        self.saddr6 = e(torch.uint8, 16) if with_v6 else None
        self.daddr6 = e(torch.uint8, 16) if with_v6 else None
        if parse:
            self.parse()

    def parse(self):
        fr = gf_frames(self.n, self.frames.shape[1] if self.n else 64, _ptr(self.frames), _ptr(self.len))
        o = gf_pkt_cols_out(_ptr(self.ethertype), _ptr(self.saddr4), _ptr(self.daddr4), _ptr(self.proto),
                            _ptr(self.l4_off), _ptr(self.l4w0), _ptr(self.l4w3), _ptr(self.saddr6),
                            _ptr(self.daddr6))
        _check(lib.gf_parse_frames(C.byref(fr), C.byref(o), _stream()), "gf_parse_frames")

    def cols(self):
        return gf_pkt_cols(self.n, _ptr(self.len), _ptr(self.ethertype), _ptr(self.saddr4), _ptr(self.daddr4),
                           _ptr(self.proto), _ptr(self.l4_off), _ptr(self.l4w0), _ptr(self.l4w3),
                           _ptr(self.saddr6), _ptr(self.daddr6), _ptr(self.src_identity), _ptr(self.ifindex),
                           _ptr(self.lxc_id), _ptr(self.tc_index), _ptr(self.flow_hash))

    def columns_numpy(self):
        torch = _torch()
        torch.cuda.synchronize()
        g = lambda t, dt: t.cpu().numpy().view(dt)
        out = {"ethertype": g(self.ethertype, np.uint16), "saddr4": g(self.saddr4, np.uint32),
               "daddr4": g(self.daddr4, np.uint32), "proto": g(self.proto, np.uint8),
               "l4_off": g(self.l4_off, np.int16), "l4w0": g(self.l4w0, np.uint32), "l4w3": g(self.l4w3, np.uint16)}
        if self.saddr6 is not None:
            out["saddr6"] = self.saddr6.cpu().numpy()
            out["daddr6"] = self.daddr6.cpu().numpy()
        return out


class Datapath:
    """Installs a synth.Scenario into libgpuflow and exposes the classify calls."""

    def __init__(self, sc, pin_prefix=""):
        self.sc = sc
        self.fd = {}
        for name, m in sc.maps.items():
            fd = bpf.CreateMap(m.type, m.ksz, m.vsz, m.max_entries, m.flags)
            if m.n():
                k = np.ascontiguousarray(m.keys, np.uint8)
                v = np.ascontiguousarray(m.vals, np.uint8)
                bpf.UpdateBatch(fd, k.ctypes.data, v.ctypes.data, m.n(), bpf.BPF_ANY)
            if pin_prefix is not None:
                try:
                    bpf.ObjPin(fd, bpf.MapPath(pin_prefix + name))
                except OSError:
                    pass
            self.fd[name] = fd
        h = lambda name: self.fd[name] if name else 0
        nd = sc.node or {}
        ncfg = gf_node_cfg(sc.host_ifindex, h(nd.get("proxy4")), h(nd.get("proxy6")), nd.get("ipv4_gateway", 0),
                           (C.c_uint8 * 16)(*nd.get("host_ip6", bytes(16))), (C.c_uint8 * 6)(*nd.get("host_mac", bytes(6))),
                           (C.c_uint8 * 6)(*nd.get("node_mac", bytes(6))), h(nd.get("lxc_map")),
                           nd.get("ipv4_cluster_range", 0), nd.get("ipv4_cluster_mask", 0), nd.get("ipv4_loopback", 0),
                           nd.get("ipv4_mask", 0), nd.get("encap_ifindex", 0), h(nd.get("tunnel_map")),
                           (C.c_uint8 * 16)(*nd.get("router_ip6", bytes(16))))
        _check(lib.gf_node_config(C.byref(ncfg)), "gf_node_config")
        self.xdp_prog = self.lb_prog = self.policy_array = None
        if sc.xdp:
            x = sc.xdp
            cfg = gf_xdp_cfg(h(x.get("cidr4_hmap")), h(x.get("cidr4_lmap")), h(x.get("cidr6_hmap")),
                             h(x.get("cidr6_lmap")), h(x.get("lxc_map")))
            self.xdp_prog = _check(lib.gf_xdp_prog_load(C.byref(cfg)), "gf_xdp_prog_load")
        if sc.lb:
            cfg = gf_lb_cfg(h(sc.lb.get("lb4")), h(sc.lb.get("lb6")), sc.lb["flags"], sc.lb.get("redirect_ifindex", 0))
            self.lb_prog = _check(lib.gf_lb_prog_load(C.byref(cfg)), "gf_lb_prog_load")
        if sc.lxc:
            self.policy_array = _check(lib.gf_policy_array_create(), "gf_policy_array_create")
            self.lxc_progs = []
            for e in sc.lxc:
                cfg = gf_lxc_cfg()
                cfg.lxc_id, cfg.seclabel = e["lxc_id"], e["seclabel"]
                cfg.policy_map, cfg.ct_map4, cfg.ct_map6 = h(e.get("policy")), h(e.get("ct4")), h(e.get("ct6"))
                cfg.cidr4_ingress_map, cfg.cidr6_ingress_map = h(e.get("cidr4")), h(e.get("cidr6"))
                cfg.revnat4_map, cfg.revnat6_map = h(e.get("revnat4")), h(e.get("revnat6"))
                cfg.flags = e["flags"]
                l4 = e.get("l4") or []
                cfg.n_l4_ingress = len(l4)
                for i, (port, proxy, nh) in enumerate(l4):
                    cfg.l4_ingress[i].port = ((port & 0xff) << 8) | (port >> 8)
                    cfg.l4_ingress[i].proxy = ((proxy & 0xff) << 8) | (proxy >> 8)
                    cfg.l4_ingress[i].nexthdr = nh
                egress_fields(cfg, e, h)
                p = _check(lib.gf_lxc_prog_load(C.byref(cfg)), "gf_lxc_prog_load")
                self.lxc_progs.append(p)
                _check(lib.gf_policy_array_update(self.policy_array, e["lxc_id"], p), "gf_policy_array_update")

        self.pipe = None
        if sc.netdev and self.policy_array:
            nd = sc.netdev
            ncfg = gf_netdev_cfg(h(nd["lxc_map"]), nd.get("flags", 0), nd.get("fixed_secctx", 0),
                                 (C.c_uint8 * 16)(*nd.get("router_ip6", bytes(16))), nd.get("ingress_ifindex", 0))
            pcfg = gf_pipeline_cfg(self.xdp_prog or 0, self.lb_prog or 0, ncfg, self.policy_array)
            self.pipe = _check(lib.gf_pipeline_load(C.byref(pcfg)), "gf_pipeline_load")

    # ---- classify calls -------------------------------------------------
    def xdp(self, b):
        torch = _torch()
        out = torch.empty(b.n, dtype=torch.uint8, device=b.device)
        c = b.cols()
        _check(lib.gf_xdp_classify(self.xdp_prog, C.byref(c), _ptr(out), _stream()), "gf_xdp_classify")
        return out

    def lb(self, b):
        torch = _torch()
        out = torch.empty((b.n, 12), dtype=torch.uint8, device=b.device)
        nd6 = torch.empty((b.n, 16), dtype=torch.uint8, device=b.device)
        c = b.cols()
        _check(lib.gf_lb_classify(self.lb_prog, C.byref(c), _ptr(out), _ptr(nd6), _stream()), "gf_lb_classify")
        return out, nd6

    def ingress(self, b, now, out=None):
        torch = _torch()
        if out is None:
            out = torch.empty((b.n, 8), dtype=torch.uint8, device=b.device)
        c = b.cols()
        _check(lib.gf_policy_ingress_classify(self.policy_array, C.byref(c), now, _ptr(out), _stream()),
               "gf_policy_ingress_classify")
        return out

    def ingress_batches(self, bs, nows, outs=None):
        """gf_policy_ingress_classify_batches: the batches in order, each batch's
        schedule built on a second stream while the previous one runs."""
        torch = _torch()
        if outs is None:
            outs = [torch.empty((b.n, 8), dtype=torch.uint8, device=b.device) for b in bs]
        cols = [b.cols() for b in bs]
        k = len(bs)
        cp = (C.POINTER(gf_pkt_cols) * k)(*[C.pointer(c) for c in cols])
        nw = (C.c_uint32 * k)(*[int(x) for x in nows])
        op = (C.c_void_p * k)(*[_ptr(o) for o in outs])
        _check(lib.gf_policy_ingress_classify_batches(self.policy_array, k, cp, nw, op, _stream()),
               "gf_policy_ingress_classify_batches")
        return outs

    def pipeline(self, b, now, out=None, snap_out=True):
        """Full pipeline over the batch's frames: returns (records [n,24] u8,
        new_daddr6 [n,16] u8, rewritten snaps [n,stride] u8 or None)."""
        torch = _torch()
        if out is None:
            out = torch.empty((b.n, 24), dtype=torch.uint8, device=b.device)
        nd6 = torch.empty((b.n, 16), dtype=torch.uint8, device=b.device)
        snap = torch.empty_like(b.frames) if snap_out else None
        stride = b.frames.shape[1] if b.n else 64
        pb = gf_pipe_batch(gf_frames(b.n, stride, _ptr(b.frames), _ptr(b.len)), _ptr(b.tc_index), _ptr(b.flow_hash))
        _check(lib.gf_pipeline_classify(self.pipe, C.byref(pb), now, _ptr(out), _ptr(nd6), _ptr(snap), _stream()),
               "gf_pipeline_classify")
        return out, nd6, snap

    def egress(self, b, now, out=None, snap_out=True):
        """The from-container program over the batch's frames (+ handle_policy of the
        local deliveries): returns (records [n,24] u8, rewritten snaps or None)."""
        torch = _torch()
        if out is None:
            out = torch.empty((b.n, 24), dtype=torch.uint8, device=b.device)
        snap = torch.empty_like(b.frames) if snap_out else None
        stride = b.frames.shape[1] if b.n else 64
        eb = gf_lxc_batch(gf_frames(b.n, stride, _ptr(b.frames), _ptr(b.len)), _ptr(b.lxc_id), _ptr(b.flow_hash))
        _check(lib.gf_lxc_egress_classify(self.policy_array, C.byref(eb), now, _ptr(out), _ptr(snap), _stream()),
               "gf_lxc_egress_classify")
        return out, snap

    # ---- map readback ----------------------------------------------------
    def dump_map(self, name):
        m = self.sc.maps[name]
        d = {}
        bpf_map = bpf.Map(name, m.type, m.ksz, m.vsz, m.max_entries, m.flags)
        bpf_map.fd = self.fd[name]
        bpf_map.DumpWithCallback(lambda k, v: d.__setitem__(k, v))
        return d

    def close(self):
        """Close the program objects, then the maps (a program holds its maps, so
        their device tables are released once both are closed)."""
        progs = [self.pipe, self.policy_array, self.lb_prog, self.xdp_prog] + list(getattr(self, "lxc_progs", []))
        for h in [h for h in progs if h] + list(self.fd.values()):
            try:
                bpf.ObjClose(h)
            except OSError:
                pass
        self.pipe = self.policy_array = self.lb_prog = self.xdp_prog = None
        self.lxc_progs = []
        self.fd = {}


def to_numpy(t, dtype):
    return t.cpu().numpy().view(dtype).reshape(-1)
