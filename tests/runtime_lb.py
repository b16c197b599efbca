"""The reference runtime suite's service load-balancing checks
(tests/golden/runtime_lb.json, test/runtime/lb.go) as datapath scenarios —
TEST INFRASTRUCTURE.

The agent's part (services -> lbmap, pkg/maps/lbmap/lbmap.go:318-369
AddSVC2BPFMap with addRevNAT): each backend is slave s = 1..n of {VIP, port}
with its target, port and rev_nat_index = the service id
(LBSVC2ServiceKeynValue, :381-410); the master {VIP, port, 0} holds count = n,
weight = the number of non-zero weights (0) and no rev_nat_index; the
reverse-NAT map holds id -> {VIP, port}.  Every endpoint program has LB_L3 and
LB_L4 (pkg/endpoint/bpf.go:279-280); no policy is loaded (AfterEach
PolicyDelAll, default enforcement), so neither direction is enforced.  The
endpoint map also holds the node's own addresses as host entries
(daemon/daemon.go:834-845: the external IPv4 10.0.2.15 of the test VM and the
router IPv6), each in the ipcache as reserved:host.

The network's part — each packet through the program the reference runs it
through:

  from a container    its from-container program (bpf_lxc.c handle_ingress,
                      lb4_local / lb6_local); a local destination continues
                      into that endpoint's handle_policy
  from the host       createLBDevice (lb.go:460-530): the host routes 2.2.2.2
                      out of lbtest1, bpf_lb on lbtest2's ingress (LB_L3,
                      LB_REDIRECT = cilium_host) translates it and redirects it
                      to cilium_host, whose egress program is bpf_netdev with
                      FROM_HOST and FIXED_SRC_SECCTX = HOST_ID (bpf/init.sh:359-360).
                      The harness plays that chain as one pipeline call whose LB
                      stage is configured without the redirect, so the translated
                      frame continues into bpf_netdev (HOST_ID) in the same call.
                      Replies of the host take the same call: bpf_lb finds no
                      service for an endpoint address and passes the frame on
                      unchanged (lb4_lookup_service -> NULL, bpf_lb.c:139-143).

A check passes when every packet of the exchange reaches the other side (ping:
echo request, echo reply; curl: SYN, SYN-ACK, ACK to the same backend) and, for
a container client, the reply it receives comes from the frontend (the
reverse NAT of handle_policy / the loopback path), as ping and curl require.
The bpf_lb path is stateless and its IPv4 reply keeps the backend's address;
the host's ping accepts it by ICMP identifier, so that leg checks delivery only.
"""
import ipaddress
import json
import os

import numpy as np

from cilium_amd import synth as S
from tests import runtime_matrix as RM

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runtime_lb.json")
HOST_ID = 1
SESSIONS = 6                      # ping / curl runs per check: own ICMP id / source port / skb hash
STRIDE = RM.STRIDE
TCP_SEQ = RM.TCP_SEQ


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def topology(doc):
    return RM.Topology({n: {"labels": [f"id.{n}"], "identity": 400 + k} for k, n in enumerate(doc["endpoints"])})


def _is_v6(a):
    return ":" in a


def addr(doc, topo, who, v6):
    """Packed address of an endpoint name, 'host' or a literal address."""
    if who == "host":
        who = doc["host6"] if v6 else doc["host4"]
    if who in topo.ip4:
        return topo.ip6[who] if v6 else S.be32_bytes([topo.ip4[who]]).tobytes()
    return ipaddress.ip_address(who).packed


def compile_case(doc, case, topo, ct_max=1 << 16):
    sc = S.Scenario("runtime-lb:" + case["name"], now=5000, host_ifindex=1)
    sc.add_map(S.MapSpec("ct4", S.LRU_HASH, 14, 48, ct_max))
    sc.add_map(S.MapSpec("ct6", S.LRU_HASH, 40, 48, ct_max))
    names = topo.names
    ip4 = np.array([topo.ip4[n] for n in names], np.uint32)
    ip6 = np.array([np.frombuffer(topo.ip6[n], np.uint8) for n in names])
    ids = np.array([topo.ident[n] for n in names], np.uint32)
    ev = S.endpoint_infos(np.array([topo.ifindex[n] for n in names], np.uint32), ids,
                          np.array([topo.lxc_id[n] for n in names], np.uint32), np.zeros(len(names)))
    ev[:, 16:22] = np.array([np.frombuffer(topo.mac[n], np.uint8) for n in names])
    ev[:, 24:30] = np.frombuffer(RM.NODE_MAC, np.uint8)
    host4 = np.array([S.ip4(doc["host4"])], np.uint32)
    host6 = np.frombuffer(RM.ROUTER6, np.uint8)[None]
    hk = np.concatenate([S.endpoint_keys4(host4), S.endpoint_keys6(host6)])
    hv = np.zeros((2, 112), np.uint8)
    hv[:, 8] = 1                                           # EndpointFlagHost (lxcmap.go:192-197)
    sc.add_map(S.MapSpec("cilium_lxc", S.HASH, 20, 112, 65535, 0,
                         np.concatenate([S.endpoint_keys4(ip4), S.endpoint_keys6(ip6), hk]),
                         np.concatenate([ev, ev, hv])))
    icv = np.zeros((len(names), 8), np.uint8)
    icv[:, 0:2] = S.le_bytes(ids, "<u2")
    hic = np.zeros((2, 8), np.uint8)
    hic[:, 0] = HOST_ID
    sc.add_map(S.MapSpec("cilium_ipcache", S.HASH, 20, 8, 512000, 0,
                         np.concatenate([S.endpoint_keys4(ip4), S.endpoint_keys6(ip6), hk]),
                         np.concatenate([icv, icv, hic])))
    # lbmap: slaves 1..n, master, reverse NAT
    k4, v4, k6, v6, r4, r6 = [], [], [], [], [], []
    for svc in case["services"]:
        fe, port = svc["frontend"]
        v6f = _is_v6(fe)
        bes = svc["backends"]
        if v6f:
            vip = np.frombuffer(ipaddress.ip_address(fe).packed, np.uint8)[None]
            tg = np.array([np.frombuffer(addr(doc, topo, b, True), np.uint8) for b, _ in bes])
            k6 += [S.lb6_keys(np.repeat(vip, len(bes), 0), [port] * len(bes), np.arange(1, len(bes) + 1)),
                   S.lb6_keys(vip, [port], [0])]
            v6 += [S.lb6_vals(tg, [p for _, p in bes], [0] * len(bes), [svc["id"]] * len(bes)),
                   S.lb6_vals(np.zeros((1, 16), np.uint8), [0], [len(bes)], [0])]
            r6.append(S.revnat6_entries([svc["id"]], vip, [port]))
        else:
            vip = S.ip4(fe)
            tg = [int.from_bytes(addr(doc, topo, b, False), "big") for b, _ in bes]
            k4 += [S.lb4_keys([vip] * len(bes), [port] * len(bes), np.arange(1, len(bes) + 1)),
                   S.lb4_keys([vip], [port], [0])]
            v4 += [S.lb4_vals(tg, [p for _, p in bes], [0] * len(bes), [svc["id"]] * len(bes)),
                   S.lb4_vals([0], [0], [len(bes)], [0])]
            r4.append(S.revnat4_entries([svc["id"]], np.array([vip], np.uint32), [port]))
    cat = lambda xs, w: np.concatenate(xs) if xs else None
    sc.add_map(S.MapSpec("lb4_svc", S.HASH, 8, 12, 65536, 0, cat(k4, 8), cat(v4, 12)))
    sc.add_map(S.MapSpec("lb6_svc", S.HASH, 20, 24, 65536, 0, cat(k6, 20), cat(v6, 24)))
    sc.add_map(S.MapSpec("revnat4", S.HASH, 2, 6, 65536, 0, cat([k for k, _ in r4], 2), cat([v for _, v in r4], 6)))
    sc.add_map(S.MapSpec("revnat6", S.HASH, 2, 18, 65536, 0, cat([k for k, _ in r6], 2), cat([v for _, v in r6], 18)))
    raw_be = lambda a: int(S.be32_bytes([a]).view("<u4")[0, 0])
    sc.node = {"lxc_map": "cilium_lxc", "ipv4_cluster_range": raw_be(S.ip4("10.0.0.0")),
               "ipv4_cluster_mask": raw_be(0xFF000000), "ipv4_loopback": raw_be(S.ip4("10.255.255.245")),
               "ipv4_mask": raw_be(0xFFFF0000), "router_ip6": RM.ROUTER6,
               "host_mac": bytes([0xce, 0x72, 0xa7, 0x03, 0x88, 0x56]), "node_mac": RM.NODE_MAC}
    for n in names:
        sc.add_map(S.MapSpec(f"pol_{n}", S.HASH, 8, 24, 16384, 0))
        sc.lxc.append({"lxc_id": topo.lxc_id[n], "seclabel": topo.ident[n], "policy": f"pol_{n}",
                       "ct4": "ct4", "ct6": "ct6", "revnat4": "revnat4", "revnat6": "revnat6",
                       "lb4": "lb4_svc", "lb6": "lb6_svc", "ipcache": "cilium_ipcache",
                       "flags": S.LXC_CT_ACCOUNTING | S.LXC_LXC_IPV4, "lxc_mac": topo.mac[n],
                       "node_mac": RM.NODE_MAC, "lxc_ipv4": raw_be(topo.ip4[n]), "lxc_ip6": topo.ip6[n]})
    sc.lb = {"lb4": "lb4_svc", "lb6": "lb6_svc", "flags": S.LB_L3, "redirect_ifindex": 0}
    sc.netdev = {"lxc_map": "cilium_lxc", "flags": 1, "fixed_secctx": HOST_ID, "router_ip6": RM.ROUTER6}
    return sc


class Flow:
    def __init__(self, j, check, session):
        self.client, self.target, self.req, self.ok = check[:4]
        self.v6 = self.req in ("ping6", "http6")
        self.tcp = self.req.startswith("http")
        self.session = session
        self.port = 80 if self.tcp else 0
        self.ident = 40000 + j                 # TCP source port / ICMP echo identifier
        self.hash = (0x9E3779B1 * (j + 1)) & 0xFFFFFFFF
        self.steps = list(TCP_SEQ) if self.tcp else [(None, "c"), (None, "s")]
        self.delivered = 0
        self.dead = False
        self.server = None                     # ("lxc", name) or ("host",)
        self.backends = set()                  # where the service may send it
        self.rx = None                         # the last frame as the receiving side got it
        self.reply_src_ok = True


def flows_of(case):
    out = []
    for check in case["checks"]:
        for s in range(SESSIONS):
            f = Flow(len(out), check, s)
            for svc in case["services"]:
                if svc["frontend"] == [f.target, f.port]:
                    f.backends = {("lxc", b) if not b[0].isdigit() and ":" not in b else ("host",)
                                  for b, _ in svc["backends"]}
            out.append(f)
    return out


def _fields(fr, v6):
    """(saddr, daddr, sport, dport) of a frame row (no IP options)."""
    if v6:
        return bytes(fr[22:38]), bytes(fr[38:54]), int.from_bytes(bytes(fr[54:56]), "big"), \
            int.from_bytes(bytes(fr[56:58]), "big")
    return bytes(fr[26:30]), bytes(fr[30:34]), int.from_bytes(bytes(fr[34:36]), "big"), \
        int.from_bytes(bytes(fr[36:38]), "big")


def _build(f, sa, da, sp, dp, flags, req_side):
    l4 = 54 if f.v6 else 34
    if f.v6:
        fr, ln = S.frames_v6(1, STRIDE, np.frombuffer(sa, np.uint8)[None], np.frombuffer(da, np.uint8)[None],
                             S.TCP if f.tcp else S.ICMPV6, sp, dp, flags or 0, 128 if req_side else 129)
    else:
        fr, ln = S.frames_v4(1, STRIDE, int.from_bytes(sa, "big"), int.from_bytes(da, "big"),
                             S.TCP if f.tcp else S.ICMP, sp, dp, flags or 0, 8 if req_side else 0)
    if not f.tcp:
        fr[0, l4 + 4:l4 + 6] = list(f.ident.to_bytes(2, "big"))      # echo identifier
    return fr, ln


def _frame(doc, topo, f, step):
    """(frame, lens, entry, lxc_id): entry 'egress' (from-container of lxc_id) or
    'pipeline' (the host side)."""
    flags, side = f.steps[step]
    if side == "c":
        sa = addr(doc, topo, f.client, f.v6)
        da = ipaddress.ip_address(f.target).packed
        fr, ln = _build(f, sa, da, f.ident, f.port, flags, True)
        src = f.client
    else:                                      # the server answers what it received
        rs, rd, rsp, rdp = _fields(f.rx, f.v6)
        fr, ln = _build(f, rd, rs, rdp, rsp, flags, False)
        src = f.server[1] if f.server[0] == "lxc" else "host"
    if src == "host":
        return fr, ln, "pipeline", 0
    fr[0, 0:6] = np.frombuffer(RM.NODE_MAC, np.uint8)
    fr[0, 6:12] = np.frombuffer(topo.mac[src], np.uint8)
    return fr, ln, "egress", topo.lxc_id[src]


def _arrival(rec, entry, topo):
    """Where a packet ended: ('lxc', name), ('host',) or None (dropped / elsewhere)."""
    if rec["action"] == 2:
        return None
    if rec["stage"] == 4:
        by_id = {v: k for k, v in topo.lxc_id.items()}
        return ("lxc", by_id.get(int(rec["lxc_id"])))
    if entry == "egress" and rec["stage"] == 5 and rec["eg_flags"] & 0x0180:    # TO_HOST | TO_STACK
        return ("host",)
    return None


def run_case(doc, case, topo, backend, now0=5000):
    """Plays every check's sessions in waves (every flow's k-th packet in wave k,
    a flow stopping at its first undelivered packet).  Returns (flows, log)."""
    flows = flows_of(case)
    log = []
    for step in range(3):
        live = [f for f in flows if not f.dead and step < len(f.steps)]
        if not live:
            break
        rows = {"egress": [], "pipeline": []}
        for f in live:
            fr, ln, entry, lid = _frame(doc, topo, f, step)
            rows[entry].append((f, fr, ln, lid))
        for entry in ("egress", "pipeline"):
            rs = rows[entry]
            if not rs:
                continue
            pk = S.Packets(np.concatenate([x[1] for x in rs]), np.concatenate([x[2] for x in rs]),
                           lxc_id=np.array([x[3] for x in rs], np.uint16),
                           flow_hash=np.array([x[0].hash for x in rs], np.uint32))
            rec, snap = getattr(backend, entry)(pk, now0 + step)
            log.append((entry, step, rec, snap))
            for i, (f, *_) in enumerate(rs):
                side = f.steps[step][1]
                where = _arrival(rec[i], entry, topo)
                if side == "c":
                    good = where in f.backends and (f.server is None or where == f.server)
                    if good:
                        f.server = where
                else:
                    want = ("host",) if f.client == "host" else ("lxc", f.client)
                    good = where == want
                    if good and f.client != "host":
                        rs_, _, rsp, _ = _fields(snap[i], f.v6)
                        f.reply_src_ok &= rs_ == ipaddress.ip_address(f.target).packed and \
                            (not f.tcp or rsp == f.port)
                f.rx = np.array(snap[i])
                f.delivered += good
                f.dead = not good
    return flows, log


def outcomes(flows):
    """{(client, target, request): [success per session]}."""
    res = {}
    for f in flows:
        res.setdefault((f.client, f.target, f.req), []).append(
            f.delivered == len(f.steps) and f.reply_src_ok)
    return res


def mismatches(case, flows):
    exp = {(c, t, r): ok for c, t, r, ok, *_ in case["checks"]}
    return [(k, exp[k], v) for k, v in outcomes(flows).items() if any(o != exp[k] for o in v)]


class OracleBackend:
    def __init__(self, sc):
        from oracle.scenario import OracleDP
        self.dp = OracleDP(sc)

    def egress(self, pk, now):
        o, snap = self.dp.egress(pk, now)
        return o, snap

    def pipeline(self, pk, now):
        o, _, snap = self.dp.pipeline(pk, now)
        return o, snap


class GpuBackend:
    """The HIP path through libgpuflow's C ABI (gf_lxc_egress_classify,
    gf_pipeline_classify), rewritten frames included."""

    def __init__(self, sc):
        from cilium_amd.datapath import Datapath
        self.dp = Datapath(sc, pin_prefix=None)

    def egress(self, pk, now):
        import torch
        from cilium_amd.datapath import DeviceBatch, EG_OUT
        out, snap = self.dp.egress(DeviceBatch(pk, parse=False), now)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(EG_OUT).ravel(), snap.cpu().numpy()

    def pipeline(self, pk, now):
        import torch
        from cilium_amd.datapath import DeviceBatch, PIPE_OUT
        out, _, snap = self.dp.pipeline(DeviceBatch(pk, parse=False), now)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(PIPE_OUT).ravel(), snap.cpu().numpy()

    def dump(self, name, ksz):
        from cilium_amd import bpf
        m = bpf.Map(name, 9, ksz, 48, 1 << 16)
        m.fd = self.dp.fd[name]
        return m.DumpArrays()

    def close(self):
        self.dp.close()
