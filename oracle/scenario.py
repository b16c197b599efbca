"""Installs a cilium_amd.synth.Scenario into the CPU oracle — TEST INFRASTRUCTURE ONLY."""
import ctypes as C

import numpy as np

from . import oracle as O


def _be16(x):
    return ((x & 0xff) << 8) | (x >> 8)


def egress_fields(c, e, h):
    """The from-container section of an endpoint config (o_lxc_cfg / gf_lxc_cfg)."""
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


class OracleDP:
    def __init__(self, sc, shards=1):
        self.sc = sc
        self.m = {}
        for name, spec in sc.maps.items():
            sh = shards if spec.ksz in (14, 40) else 1
            om = O.OMap(spec.type, spec.ksz, spec.vsz, spec.max_entries, sh)
            if spec.n():
                om.update_many(np.ascontiguousarray(spec.keys, np.uint8), np.ascontiguousarray(spec.vals, np.uint8))
            self.m[name] = om
        p = lambda name: self.m[name].ptr if name else None
        nd = sc.node or {}
        self._node = O.o_node_cfg(sc.host_ifindex, p(nd.get("proxy4")), p(nd.get("proxy6")), nd.get("ipv4_gateway", 0),
                                  (C.c_uint8 * 16)(*nd.get("host_ip6", bytes(16))),
                                  (C.c_uint8 * 6)(*nd.get("host_mac", bytes(6))),
                                  (C.c_uint8 * 6)(*nd.get("node_mac", bytes(6))),
                                  p(nd.get("lxc_map")), nd.get("ipv4_cluster_range", 0), nd.get("ipv4_cluster_mask", 0),
                                  nd.get("ipv4_loopback", 0), nd.get("ipv4_mask", 0), nd.get("encap_ifindex", 0),
                                  p(nd.get("tunnel_map")), (C.c_uint8 * 16)(*nd.get("router_ip6", bytes(16))))
        O.lib.o_set_node(C.byref(self._node))
        self.xdp_cfg = self.lb_cfg = None
        if sc.xdp:
            x = sc.xdp
            self.xdp_cfg = O.o_xdp_cfg(p(x.get("cidr4_hmap")), p(x.get("cidr4_lmap")), p(x.get("cidr6_hmap")),
                                       p(x.get("cidr6_lmap")), p(x.get("lxc_map")))
        if sc.lb:
            self.lb_cfg = O.o_lb_cfg(p(sc.lb.get("lb4")), p(sc.lb.get("lb6")), sc.lb["flags"],
                                     sc.lb.get("redirect_ifindex", 0))
        self.arr = None
        self._pipe = None
        self.cfgs = []
        # LRU stand-in: the CT maps the programs bind, each with its
        # classify-call counter; lru_replay[name] = {seq: (age_cut, hand, lines)} replays
        # the GPU's logged evictions instead (a sampled run holds only part of the table)
        self.lru_maps = sorted({e[k] for e in sc.lxc for k in ("ct4", "ct6") if e.get(k)
                                and sc.maps[e[k]].type == 9})
        self.lru_seq = {n: 0 for n in self.lru_maps}
        self.lru_replay = {}
        self.lru_log = {n: [] for n in self.lru_maps}
        if sc.lxc:
            self.arr = O.lib.o_prog_array_create()
            for e in sc.lxc:
                c = O.o_lxc_cfg()
                c.lxc_id, c.seclabel = e["lxc_id"], e["seclabel"]
                c.policy_map, c.ct_map4, c.ct_map6 = p(e.get("policy")), p(e.get("ct4")), p(e.get("ct6"))
                c.cidr4_ingress_map, c.cidr6_ingress_map = p(e.get("cidr4")), p(e.get("cidr6"))
                c.revnat4_map, c.revnat6_map = p(e.get("revnat4")), p(e.get("revnat6"))
                c.flags = e["flags"]
                l4 = e.get("l4") or []
                c.n_l4_ingress = len(l4)
                for i, (port, proxy, nh) in enumerate(l4):
                    c.l4_ingress[i].port = ((port & 0xff) << 8) | (port >> 8)
                    c.l4_ingress[i].proxy = ((proxy & 0xff) << 8) | (proxy >> 8)
                    c.l4_ingress[i].nexthdr = nh
                egress_fields(c, e, p)
                self.cfgs.append(c)
                O.lib.o_prog_array_set(self.arr, e["lxc_id"], C.byref(c))

    @staticmethod
    def batch(pk):
        return O.make_batch(pk.frames, pk.lens, pk.src_identity, pk.ifindex, pk.lxc_id, pk.tc_index, pk.flow_hash)

    def parse(self, pk):
        return O.parse(self.batch(pk))

    def xdp(self, pk, threads=1):
        return O.xdp(self.xdp_cfg, self.batch(pk), threads)

    def lb(self, pk, threads=1):
        return O.lb(self.lb_cfg, self.batch(pk), threads)

    def lru_after_call(self, now):
        """After every classify call: the LRU stand-in on each bound CT map."""
        for n in self.lru_maps:
            self.lru_seq[n] += 1
            seq = self.lru_seq[n]
            if n in self.lru_replay:
                e = self.lru_replay[n].get(seq)
                if e is not None:
                    ev = self.m[n].lru_replay(now, *e)
                    self.lru_log[n].append((seq, now) + tuple(e) + (ev,))
            else:
                r = self.m[n].lru_evict(now)
                if r is not None:
                    self.lru_log[n].append((seq, now) + r)

    def ingress(self, pk, now, threads=1, lru=True):
        """handle_policy over the batch; lru=False: part of a call whose LRU step
        comes with its last part (a batch split across calls)."""
        O.lib.o_set_node(C.byref(self._node))           # node_config.h is per thread in the restatement
        out = O.ingress(self.arr, self.batch(pk), now, threads)
        if lru:
            self.lru_after_call(now)
        return out

    def ingress_events(self, pk, out):
        return O.ingress_events(self.arr, self.batch(pk), out)

    def pipeline(self, pk, now, threads=1, events=False, lru=True):
        O.lib.o_set_node(C.byref(self._node))
        if self._pipe is None:
            nd = self.sc.netdev
            self._nd = O.o_netdev_cfg(self.m[nd["lxc_map"]].ptr, nd.get("flags", 0), nd.get("fixed_secctx", 0),
                                      (C.c_uint8 * 16)(*nd.get("router_ip6", bytes(16))), nd.get("ingress_ifindex", 0))
            self._pipe = O.o_pipeline_cfg(C.pointer(self.xdp_cfg) if self.xdp_cfg is not None else None,
                                          C.pointer(self.lb_cfg) if self.lb_cfg is not None else None,
                                          C.pointer(self._nd), self.arr)
        r = O.pipeline(self._pipe, self.batch(pk), now, threads, events)
        if lru:
            self.lru_after_call(now)
        return r

    def egress(self, pk, now, events=False):
        O.lib.o_set_node(C.byref(self._node))
        r = O.egress(self.arr, self.batch(pk), now, events)
        self.lru_after_call(now)
        return r

    def ct_gc(self, name, filter_time):
        return self.m[name].ct_gc(filter_time)

    def dump(self, name):
        return self.m[name].dump()

    def __del__(self):
        try:
            if self.arr:
                O.lib.o_prog_array_destroy(self.arr)
                self.arr = None
        except Exception:
            pass
