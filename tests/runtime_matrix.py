"""The reference runtime suite's connectivity matrices (tests/golden/runtime_policies.json)
as datapath scenarios — TEST INFRASTRUCTURE.

A case names endpoints (labels, identity), the policy rules imported and the
client -> server requests with their expected outcome.  This module plays the
agent's part for it — rules -> per-endpoint policy map, CIDR maps and
enforcement flags — and the network's part — a request -> the packets curl /
ping put on the wire, each through the program the reference runs it through:

  request / TCP ACK      from-container program of the client (bpf_lxc.c
                         handle_ingress); a local server continues into its
                         handle_policy (ipv4_local_delivery tail call)
  reply from an endpoint from-container program of the server, then the
                         client's handle_policy
  reply from the host    the client's handle_policy entered from bpf_netdev
                         with secctx WORLD_ID (bpf_netdev.c:250-260,
                         derive_ipv4_sec_ctx without FIXED_SRC_SECCTX)

Agent restatement (pkg/ citations against /root/reference):
  enforcement        daemon/policy.go:56-75 (always: both directions; default:
                     a direction is enforced when a rule selecting the endpoint
                     has rules in it, pkg/policy/repository.go:569-588
                     GetRulesMatching) -> POLICY_INGRESS / POLICY_EGRESS
                     (pkg/endpoint/policy.go:820-839, endpoint.go:148-156)
  L3 identities      pkg/endpoint/policy.go:475-520 regenerateConsumable over
                     every identity of the cache incl. the reserved ones
                     (getLabelsMap :299-313): allowed when a selecting rule's
                     fromEndpoints/toEndpoints matches and the rule has no toPorts
                     (pkg/policy/rule.go:296-384 canReachIngress/Egress); each
                     allowed identity is a {id, 0, 0, dir} policy entry
                     (pkg/policy/consumer.go:171-247 addToPolicyMaps).
                     alwaysAllowLocalhost is false outside Kubernetes
                     (daemon/main.go:580-585, daemon.go:957-962).
  L4 filters         pkg/endpoint/policy.go:87-101, 176-217 applyNewFilter: one
                     {id, port, proto, dir} entry per identity the filter's
                     selectors match; no fromEndpoints = wildcard selector = every
                     identity.  HAVE_L4_POLICY whenever the L4 policy exists
                     (pkg/endpoint/bpf.go:135-154), CFG_L3L4_* = the filters'
                     (port, redirect, proto) without L7 redirects.
  CIDR maps          fromCIDR / toCIDR prefixes of the selecting rules
                     (pkg/policy/repository.go ResolveCIDRPolicy), a CIDR*_MAP
                     defined only when it holds prefixes (pkg/endpoint/bpf.go:252-266).
  ipcache            every endpoint address -> its identity (the host addresses are
                     removed from the endpoint map by the test, Policies.go:740-741).
"""
import ipaddress
import json
import os

import numpy as np

from cilium_amd import synth as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runtime_policies.json")
RESERVED = {1: "reserved:host", 2: "reserved:world", 3: "reserved:cluster", 4: "reserved:health"}
WORLD_ID = 2
HOST4, HOST6 = "192.168.254.254", "fdff::ff"          # test/helpers/cons.go IPv4Host / IPv6Host
NODE_MAC = bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])
ROUTER6 = ipaddress.IPv6Address("f00d::a0f:0:0:1").packed
TCP_SEQ = ((S.F_SYN, "c"), (S.F_SYN | S.F_ACK, "s"), (S.F_ACK, "c"))
REQ_ORDER = ("ping", "ping6", "http", "http6", "httpPrivate", "http6Private")
STRIDE = 128


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def case_endpoints(doc, case):
    """A case's endpoints: its own set when it names one (the conntrack suite's
    containers), else the document's."""
    return case.get("endpoints") or doc["endpoints"]


class Topology:
    """Endpoints of the runtime suite: IPv4 10.15.0.<lxc_id>, IPv6
    f00d::a0f:0:0:<lxc_id> (inside ROUTER_IP's /64 and the IPv6Gateway/112 the
    CIDR case names), one MAC each, ifindex 20 + k."""

    def __init__(self, eps):
        self.names = list(eps)
        self.ident = {n: eps[n]["identity"] for n in self.names}
        self.labels = {n: set(eps[n]["labels"]) for n in self.names}
        k = {n: i for i, n in enumerate(self.names)}
        self.lxc_id = {n: 100 + k[n] for n in self.names}
        self.ifindex = {n: 20 + k[n] for n in self.names}
        self.ip4 = {n: S.ip4("10.15.0.0") + self.lxc_id[n] for n in self.names}
        self.ip6 = {n: ipaddress.IPv6Address(int(ipaddress.IPv6Address("f00d::a0f:0:0:0")) + self.lxc_id[n]).packed
                    for n in self.names}
        self.mac = {n: bytes([0x0a, 0x00, 0x00, 0x00, 0x00, self.lxc_id[n]]) for n in self.names}
        # the identity cache: reserved identities + the endpoints'
        self.cache = {i: {l} for i, l in RESERVED.items()}
        self.cache.update({self.ident[n]: self.labels[n] for n in self.names})

    def addr(self, who, v6):
        if who == "host4":
            return S.ip4(HOST4)
        if who == "host6":
            return ipaddress.IPv6Address(HOST6).packed
        return self.ip6[who] if v6 else self.ip4[who]


def _matches(sel, labels):
    return sel == "*" or sel in labels


def _prefix(s):
    n = ipaddress.ip_network(s, strict=False)
    return n.version, n.prefixlen, n.network_address.packed


def compile_case(case, topo, ct_max=1 << 16):
    """The agent's output for one case: a synth.Scenario (maps + endpoint configs)."""
    sc = S.Scenario("runtime:" + case["name"], now=5000, host_ifindex=1)
    rules = case["rules"]
    always = case["enforcement"] == "always"
    sc.add_map(S.MapSpec("ct4", S.LRU_HASH, 14, 48, ct_max))
    sc.add_map(S.MapSpec("ct6", S.LRU_HASH, 40, 48, ct_max))
    # endpoints with the ConntrackLocal option: CT maps of their own (pkg/endpoint/bpf.go:268-276)
    local = set(case.get("conntrack_local", []))
    for n in sorted(local):
        sc.add_map(S.MapSpec(f"ct4_{n}", S.LRU_HASH, 14, 48, ct_max))
        sc.add_map(S.MapSpec(f"ct6_{n}", S.LRU_HASH, 40, 48, ct_max))
    names = topo.names
    ip4 = np.array([topo.ip4[n] for n in names], np.uint32)
    ip6 = np.array([np.frombuffer(topo.ip6[n], np.uint8) for n in names])
    ids = np.array([topo.ident[n] for n in names], np.uint32)
    lxc = np.array([topo.lxc_id[n] for n in names], np.uint32)
    ifx = np.array([topo.ifindex[n] for n in names], np.uint32)
    ev = S.endpoint_infos(ifx, ids, lxc, np.zeros(len(names)))
    ev[:, 16:22] = np.array([np.frombuffer(topo.mac[n], np.uint8) for n in names])
    ev[:, 24:30] = np.frombuffer(NODE_MAC, np.uint8)
    sc.add_map(S.MapSpec("cilium_lxc", S.HASH, 20, 112, 65535, 0,
                         np.concatenate([S.endpoint_keys4(ip4), S.endpoint_keys6(ip6)]), np.concatenate([ev, ev])))
    icv = np.zeros((len(names), 8), np.uint8)
    icv[:, 0:2] = S.le_bytes(ids, "<u2")
    sc.add_map(S.MapSpec("cilium_ipcache", S.HASH, 20, 8, 512000, 0,
                         np.concatenate([S.endpoint_keys4(ip4), S.endpoint_keys6(ip6)]), np.concatenate([icv, icv])))
    raw_be = lambda a: int(S.be32_bytes([a]).view("<u4")[0, 0])
    sc.node = {"lxc_map": "cilium_lxc", "ipv4_cluster_range": raw_be(S.ip4("10.0.0.0")),
               "ipv4_cluster_mask": raw_be(0xFF000000), "ipv4_loopback": raw_be(S.ip4("10.255.255.245")),
               "ipv4_mask": raw_be(0xFFFF0000), "router_ip6": ROUTER6,
               "host_mac": bytes([0xce, 0x72, 0xa7, 0x03, 0x88, 0x56]), "node_mac": NODE_MAC}
    state = {}
    for n in names:
        L = topo.labels[n]
        sel = [r for r in rules if any(_matches(s, L) for s in [r["select"]])]
        ing_rules = [x for r in sel for x in r.get("ingress", [])]
        eg_rules = [x for r in sel for x in r.get("egress", [])]
        pol_in = always or any(r.get("ingress") for r in sel)
        pol_eg = always or any(r.get("egress") for r in sel)
        entries = {}                                   # (identity, port, proto, egress) -> proxy port
        for d, rl, key in ((0, ing_rules, "fromEndpoints"), (1, eg_rules, "toEndpoints")):
            for ident, lab in topo.cache.items():     # L3: canReach* with no toPorts
                if any(not r.get("toPorts") and any(_matches(s, lab) for s in r.get(key, [])) for r in rl):
                    entries[(ident, 0, 0, d)] = 0
            filt = {}                                   # L4 filters, merged per (port, proto)
            for r in rl:
                for port, proto in r.get("toPorts", []):
                    pr = {"tcp": S.TCP, "udp": S.UDP}[proto]
                    sels = r.get(key)
                    cur = filt.get((port, pr), [])
                    filt[(port, pr)] = None if (cur is None or not sels) else cur + list(sels)
            for (port, pr), sels in filt.items():
                for ident, lab in topo.cache.items():
                    if sels is None or any(_matches(s, lab) for s in sels):
                        entries[(ident, port, pr, d)] = 0
            state[(n, d)] = sorted(filt)
        if entries:
            k = np.array(sorted(entries), np.uint32)
            pk = S.policy_keys(k[:, 0], k[:, 1], k[:, 2], k[:, 3].astype(np.uint8))
            pv = S.policy_vals(np.zeros(len(k)))
        else:
            pk, pv = np.zeros((0, 8), np.uint8), np.zeros((0, 24), np.uint8)
        sc.add_map(S.MapSpec(f"pol_{n}", S.HASH, 8, 24, 16384, 0, pk if len(pk) else None, pv if len(pv) else None))
        ct4, ct6 = (f"ct4_{n}", f"ct6_{n}") if n in local else ("ct4", "ct6")
        cfg = {"lxc_id": topo.lxc_id[n], "seclabel": topo.ident[n], "policy": f"pol_{n}", "ct4": ct4, "ct6": ct6,
               "flags": S.LXC_HAVE_L4_POLICY | S.LXC_CT_ACCOUNTING | S.LXC_LXC_IPV4
               | (S.LXC_POLICY_INGRESS if pol_in else 0) | (S.LXC_POLICY_EGRESS if pol_eg else 0),
               "lxc_mac": topo.mac[n], "node_mac": NODE_MAC, "lxc_ipv4": raw_be(topo.ip4[n]),
               "lxc_ip6": topo.ip6[n], "ipcache": "cilium_ipcache",
               "l4": [(p, 0, pr) for p, pr in state[(n, 0)]][:64], "l4e": [(p, 0, pr) for p, pr in state[(n, 1)]][:64]}
        for d, rl, key in ((0, ing_rules, "fromCIDR"), (1, eg_rules, "toCIDR")):
            pfx = [_prefix(c) for r in rl for c in r.get(key, [])]
            for ver, bits, kf in ((4, 32, S.lpm4_keys), (6, 128, S.lpm6_keys)):
                sel_p = [(pl, net) for v, pl, net in pfx if v == ver]
                if not sel_p:
                    continue
                pl = np.array([p for p, _ in sel_p], np.uint32)
                net = (np.array([int.from_bytes(x, "big") for _, x in sel_p], np.uint32) if ver == 4
                       else np.array([np.frombuffer(x, np.uint8) for _, x in sel_p]))
                ck, cv = S.lpm_dedup(kf(pl, net), np.ones((len(pl), 1), np.uint8), bits)
                mname = f"cidr{ver}{'ie'[d]}_{n}"
                sc.add_map(S.MapSpec(mname, S.LPM, 4 + bits // 8, 1, 1024, S.NO_PREALLOC, ck, cv))
                cfg[{(4, 0): "cidr4", (6, 0): "cidr6", (4, 1): "cidr4e", (6, 1): "cidr6e"}[(ver, d)]] = mname
        sc.lxc.append(cfg)
    return sc


def expand(case):
    """[(client, server, request)] in the reference's order."""
    out = []
    for client, server, reqs, ok in case["checks"]:
        rl = list(REQ_ORDER) if reqs == "all" else reqs
        out += [(client, server, r, ok) for r in rl]
    return out


class Flow:
    """One request: ping / ping6 (ICMP echo + reply), http / http6 (TCP handshake to
    port 80), or tcp:P / tcp6:P (TCP handshake to port P) and udp:P / udp6:P (a
    datagram to port P and its reply)."""

    def __init__(self, j, client, server, req):
        self.client, self.server, self.req = client, server, req
        kind, _, port = req.partition(":")
        self.v6 = kind in ("ping6", "http6", "http6Private", "tcp6", "udp6")
        self.tcp = kind.startswith("http") or kind.startswith("tcp")
        self.udp = kind.startswith("udp")
        self.dport = int(port) if port else 80
        self.sport = 40000 + j
        self.steps = list(TCP_SEQ) if self.tcp else [(None, "c"), (None, "s")]
        self.delivered = 0                   # packets of the sequence that got through
        self.dead = False


def _frame(topo, f, step):
    flags, side = f.steps[step]
    src, dst = (f.client, f.server) if side == "c" else (f.server, f.client)
    sa, da = topo.addr(src, f.v6), topo.addr(dst, f.v6)
    sp, dp = (f.sport, f.dport) if side == "c" else (f.dport, f.sport)
    if f.v6:
        fr, ln = S.frames_v6(1, STRIDE, np.frombuffer(sa, np.uint8)[None], np.frombuffer(da, np.uint8)[None],
                             S.TCP if f.tcp else S.UDP if f.udp else S.ICMPV6, sp, dp, flags or 0,
                             128 if side == "c" else 129)
    else:
        fr, ln = S.frames_v4(1, STRIDE, sa, da, S.TCP if f.tcp else S.UDP if f.udp else S.ICMP, sp, dp, flags or 0,
                             8 if side == "c" else 0)
    if src in topo.mac:
        fr[0, 6:12] = np.frombuffer(topo.mac[src], np.uint8)
    fr[0, 0:6] = np.frombuffer(NODE_MAC, np.uint8)
    return fr, ln, src, dst


def run_case(case, topo, backend):
    """Plays the case's requests through `backend` (egress(pk, now) -> EG_OUT
    records, ingress(pk, now) -> ING_OUT records) in waves: every flow's k-th
    packet in wave k, a flow stopping at its first dropped packet (the client
    gives up).  Returns ({(client, server, request): delivered?}, per-wave records)."""
    flows = [Flow(j, c, s, r) for j, (c, s, r, _) in enumerate(expand(case))]
    log = []
    for step in range(3):
        live = [f for f in flows if not f.dead and step < len(f.steps)]
        if not live:
            break
        eg, ing = [], []
        for f in live:
            fr, ln, src, dst = _frame(topo, f, step)
            (ing if src.startswith("host") else eg).append((f, fr, ln, src, dst))
        now = case.get("now", 5000) + step
        if eg:
            pk = S.Packets(np.concatenate([x[1] for x in eg]), np.concatenate([x[2] for x in eg]),
                           lxc_id=np.array([topo.lxc_id[x[3]] for x in eg], np.uint16))
            r = backend.egress(pk, now)
            log.append(("egress", step, r))
            for (f, *_), rec in zip(eg, r):
                ok = rec["stage"] in (4, 5) and rec["action"] != 2
                f.delivered += ok
                f.dead = not ok
        if ing:
            pk = S.Packets(np.concatenate([x[1] for x in ing]), np.concatenate([x[2] for x in ing]),
                           src_identity=np.full(len(ing), WORLD_ID, np.uint32),
                           ifindex=np.array([topo.ifindex[x[4]] for x in ing], np.uint32),
                           lxc_id=np.array([topo.lxc_id[x[4]] for x in ing], np.uint16),
                           tc_index=np.zeros(len(ing), np.uint8))
            r = backend.ingress(pk, now)
            log.append(("ingress", step, r))
            for (f, *_), rec in zip(ing, r):
                ok = rec["action"] != 2
                f.delivered += ok
                f.dead = not ok
    res = {}
    for f in flows:
        res.setdefault((f.client, f.server, f.req), []).append(f.delivered == len(f.steps))
    return res, log


def run_case_one_batch(case, topo, backend):
    """Every packet of every request in ONE from-container batch, in wave order
    (all first packets, then all replies, then the ACKs): a reply shares the batch
    with its request, so its CT lookup must see the entry the request's
    handle_policy created — the per-packet order of the reference.  Only for
    cases whose servers are endpoints.  Returns (outcomes, records)."""
    flows = [Flow(j, c, s, r) for j, (c, s, r, _) in enumerate(expand(case))]
    assert not any(f.server.startswith("host") for f in flows)
    rows = []
    for step in range(3):
        for f in flows:
            if step < len(f.steps):
                fr, ln, src, _ = _frame(topo, f, step)
                rows.append((f, fr, ln, src))
    pk = S.Packets(np.concatenate([x[1] for x in rows]), np.concatenate([x[2] for x in rows]),
                   lxc_id=np.array([topo.lxc_id[x[3]] for x in rows], np.uint16))
    r = backend.egress(pk, case.get("now", 5000))
    for (f, *_), rec in zip(rows, r):
        f.delivered += rec["stage"] in (4, 5) and rec["action"] != 2
    res = {}
    for f in flows:
        res.setdefault((f.client, f.server, f.req), []).append(f.delivered == len(f.steps))
    return res, r


def expected(case):
    return {(c, s, r): ok for c, s, r, ok in expand(case)}


def outcome_mismatches(case, res):
    exp = expected(case)
    bad = []
    for k, oks in res.items():
        if any(o != exp[k] for o in oks):
            bad.append((k, exp[k], oks))
    return bad


class OracleBackend:
    def __init__(self, sc):
        from oracle.scenario import OracleDP
        self.dp = OracleDP(sc)

    def egress(self, pk, now):
        return self.dp.egress(pk, now)[0]

    def ingress(self, pk, now):
        return self.dp.ingress(pk, now)


class GpuBackend:
    """The HIP path through libgpuflow's C ABI (gf_lxc_egress_classify,
    gf_policy_ingress_classify)."""

    def __init__(self, sc):
        from cilium_amd.datapath import Datapath
        self.dp = Datapath(sc, pin_prefix=None)

    def egress(self, pk, now):
        import torch
        from cilium_amd.datapath import DeviceBatch, EG_OUT
        out, _ = self.dp.egress(DeviceBatch(pk, parse=False), now, snap_out=False)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(EG_OUT).ravel()

    def ingress(self, pk, now):
        import torch
        from cilium_amd.datapath import DeviceBatch, ING_OUT
        out = self.dp.ingress(DeviceBatch(pk), now)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(ING_OUT).ravel()

    def dump(self, name, ksz):
        from cilium_amd import bpf
        m = bpf.Map(name, 9, ksz, 48, 1 << 16)
        m.fd = self.dp.fd[name]
        return m.DumpArrays()

    def close(self):
        self.dp.close()
