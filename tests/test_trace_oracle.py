"""Hand-derived known answers for the trace notifications the oracle restates
(send_trace_notify, bpf/lib/trace.h:59-106, TRACE_NOTIFY defined for the
endpoint: pkg/endpoint/endpoint.go:131-134), read off the call sites of the
from-container program (bpf_lxc.c:650,669,705, lib/lxc.h:116, lib/encap.h:67)
and handle_policy (bpf_lxc.c:1013-1016).  Scenario: tests/test_egress_oracle.py."""
import struct

import numpy as np

import oracle.oracle as O
from cilium_amd import synth
from cilium_amd.synth import ip4, TCP, F_SYN
from oracle.scenario import OracleDP
from test_egress_oracle import _scn, _pk, S, PEER, VIP, VIP2, WORLD, TUN, NOW, LXC_MAC

TO_LXC, TO_PROXY, TO_HOST, TO_STACK, TO_OVERLAY, FROM_LXC = 0, 1, 2, 3, 4, 5


def _traced(sc, which=(0, 1)):
    for k in which:
        sc.lxc[k]["flags"] |= synth.LXC_TRACE_NOTIFY
    return sc


def _run(sc, pk, now=NOW):
    ref = OracleDP(sc)
    with O.TraceSink(pk.n) as ts:
        o, snap = ref.egress(pk, now)
    return o, snap, ts.events()


def _hdr(ev):
    """struct trace_notify / drop_notify header fields."""
    t, sub, src16, h, lo, lc, s, d = struct.unpack("<BBHIIIII", bytes(ev[:24]))
    if t == 4:
        dst_id, reason, pad, ifx = struct.unpack("<HBBI", bytes(ev[24:32]))
        return dict(type=t, obs=sub, source=src16, hash=h, len=lo, cap=lc, src=s, dst=d, dst_id=dst_id,
                    reason=reason, ifindex=ifx)
    dst_id, ifx = struct.unpack("<II", bytes(ev[24:32]))
    return dict(type=t, reason=sub, source=src16, len=lo, cap=lc, src=s, dst=d, dst_id=dst_id, ifindex=ifx)


def test_world_syn_from_lxc_then_to_stack():
    """handle_ingress traces every frame first (TRACE_FROM_LXC, SECLABEL, the frame
    as sent); pass_to_stack traces after ipv4_l3 (TRACE_TO_STACK, dstID = WORLD_ID
    outside IPV4_CLUSTER_RANGE, reason = forwarding_reason = CT_NEW)."""
    pk = _pk(WORLD, 443)
    o, snap, ev = _run(_traced(_scn()), pk)
    n = int(pk.lens[0])
    assert len(ev) == 2
    a, b = _hdr(ev[0]), _hdr(ev[1])
    assert (a["type"], a["obs"], a["source"], a["src"], a["dst"], a["ifindex"]) == (4, FROM_LXC, 100, 300, 0, 0)
    assert (a["len"], a["cap"]) == (n, min(n, 128))
    assert bytes(ev[0, 32:32 + n]) == bytes(pk.frames[0, :n])          # the frame as sent (TTL 64)
    assert (b["obs"], b["src"], b["dst"], b["dst_id"], b["ifindex"], b["reason"]) == (TO_STACK, 300, 2, 0, 0, 0)
    assert bytes(ev[1, 32:32 + n]) == bytes(snap[0, :n]) and ev[1, 32 + 22] == 63   # after ipv4_l3


def test_cluster_destination_to_stack_reports_cluster_id():
    """dstID = CLUSTER_ID when orig_dip & IPV4_CLUSTER_MASK == IPV4_CLUSTER_RANGE
    (bpf_lxc.c:509-510), reported as the TO_STACK dst_label (:669)."""
    o, snap, ev = _run(_traced(_scn()), _pk(ip4("10.200.0.9"), 443))
    assert o[0]["eg_flags"] & 0x0100
    assert [(_hdr(e)["obs"], _hdr(e)["dst"]) for e in ev] == [(FROM_LXC, 0), (TO_STACK, 3)]


def test_tunnel_to_overlay():
    """__encap_and_redirect_with_nodeid: TRACE_TO_OVERLAY(seclabel, 0, 0, ENCAP_IFINDEX, 0)."""
    o, snap, ev = _run(_traced(_scn()), _pk(TUN, 80))
    b = _hdr(ev[1])
    assert len(ev) == 2 and (b["obs"], b["src"], b["dst"], b["ifindex"], b["reason"]) == (TO_OVERLAY, 300, 0, 5, 0)


def test_local_delivery_to_lxc_of_the_destination():
    """lb4_local to the peer's backend, ipv4_local_delivery, then the destination's
    handle_policy: TRACE_TO_LXC(src_label = the sender's SECLABEL, SECLABEL, LXC_ID,
    ifindex = ep->ifindex, CT_NEW), EVENT_SOURCE = the destination's LXC_ID."""
    o, snap, ev = _run(_traced(_scn()), _pk(VIP2, 80))
    assert o[0]["stage"] == 4 and o[0]["action"] == 7
    a, b = _hdr(ev[0]), _hdr(ev[1])
    assert len(ev) == 2 and a["obs"] == FROM_LXC
    assert (b["obs"], b["source"], b["src"], b["dst"], b["dst_id"], b["ifindex"], b["reason"]) == \
        (TO_LXC, 101, 300, 301, 101, 21, 0)
    n = int(b["len"])
    assert bytes(ev[1, 32:32 + n]) == bytes(snap[0, :n])


def test_destination_without_trace_notify_sends_none():
    """TRACE_NOTIFY is per endpoint: the traced sender's FROM_LXC only."""
    o, snap, ev = _run(_traced(_scn(), which=(0,)), _pk(VIP2, 80))
    assert [_hdr(e)["obs"] for e in ev] == [FROM_LXC]
    o, snap, ev = _run(_scn(), _pk(WORLD, 443))
    assert len(ev) == 0


def test_loopback_to_sender_established():
    """The loopback service path delivers back to the sender, whose handle_policy
    finds the loopback entry (CT_ESTABLISHED) and traces TO_LXC with reason 1."""
    o, snap, ev = _run(_traced(_scn()), _pk(VIP, 80))
    b = _hdr(ev[1])
    assert (b["obs"], b["source"], b["src"], b["dst"], b["dst_id"], b["reason"]) == (TO_LXC, 100, 300, 300, 100, 1)


def test_drop_after_from_lxc():
    """A from-container drop (is_valid_lxc_src_mac -> DROP_INVALID_SMAC) comes after
    handle_ingress's FROM_LXC: the drop record is the packet's last."""
    o, snap, ev = _run(_traced(_scn()), _pk(WORLD, 80, smac=bytes(6)))
    assert [(_hdr(e)["type"]) for e in ev] == [4, 1]
    assert _hdr(ev[1])["reason"] == 130 and _hdr(ev[1])["src"] == 300


def test_egress_proxy_redirect_traced_before_rewrite():
    """ipv4_redirect_to_host_port (lib/lxc.h:96-142): TRACE_TO_PROXY(SECLABEL, 0, 0,
    HOST_IFINDEX, forwarding_reason) is sent before l4_modify_port / the daddr
    store, so its capture is the frame as the policy saw it; the redirect to the
    host that follows sends no TO_HOST."""
    sc = _scn(policy_egress=True)
    M = synth.MapSpec
    sc.maps["pol0"] = M("pol0", synth.HASH, 8, 24, 1024, 0, synth.policy_keys([2], [443], [TCP], egress=1),
                        synth.policy_vals([8080]))
    pk = _pk(WORLD, 443)
    o, snap, ev = _run(_traced(sc), pk)
    assert o[0]["eg_flags"] & 0x0002 and o[0]["action"] == 7
    n = int(pk.lens[0])
    b = _hdr(ev[1])
    assert len(ev) == 2 and (b["obs"], b["src"], b["ifindex"], b["reason"]) == (TO_PROXY, 300, 3, 0)
    assert bytes(ev[1, 32:32 + n]) == bytes(pk.frames[0, :n])          # dport 443, daddr WORLD: not yet rewritten
    assert bytes(snap[0, :n]) != bytes(pk.frames[0, :n])


def test_fuzz_event_lists_are_consistent():
    """Every packet of a traced sender starts with FROM_LXC; drops are last and only
    for SHOT packets; TO_LXC only for local deliveries that were not dropped."""
    sc = synth.egress_fuzz(seed=5, n_packets=4000, n_batches=1, hazard=False)
    for e in sc.lxc:
        e["flags"] |= synth.LXC_TRACE_NOTIFY
    ref = OracleDP(sc)
    pk = sc.batches[0]
    with O.TraceSink(pk.n) as ts:
        o, _ = ref.egress(pk, sc.now)
    has_prog = np.array([lid in {e["lxc_id"] for e in sc.lxc} for lid in pk.lxc_id])
    assert np.all(ts.cnt[has_prog] >= 1) and np.all(ts.ev[has_prog, 0, 1] == FROM_LXC)
    last = ts.ev[np.arange(pk.n), np.maximum(ts.cnt.astype(int) - 1, 0)]
    shot = o["action"] == 2
    assert np.all(last[shot & has_prog, 0] == 1) and np.all(last[~shot & has_prog, 0] == 4)
    to_lxc = (ts.ev[:, :, 0] == 4) & (ts.ev[:, :, 1] == TO_LXC)
    assert np.all(o["stage"][to_lxc.any(axis=1)] == 4) and to_lxc.sum() > 50
