"""Service load-balancing checks of the reference runtime suite (test/runtime/lb.go
RuntimeValidatedLB; tests/golden/runtime_lb.json) replayed as packets: the CPU
oracle must make every ping / curl the reference expects to succeed succeed
(request to a backend of the service, reply back, reply from the frontend),
and the HIP path must produce the oracle's records, rewritten frames and CT
tables bit-for-bit on the same packets."""
import copy

import numpy as np
import pytest

from tests import runtime_lb as RL

DOC = RL.load()
CASES = DOC["cases"]


def test_fixture_covers_reference_checks():
    assert [c["name"] for c in CASES] == ["L3 services", "L3 loopback services", "L4 services"]
    reqs = {(c, r) for case in CASES for c, _, r, *_ in case["checks"]}
    assert {("host", "ping"), ("client", "ping"), ("client", "ping6"), ("httpd1", "ping"),
            ("client", "http"), ("client", "http6")} <= reqs
    assert all(ok for case in CASES for _, _, _, ok, *_ in case["checks"])


def test_agent_restatement_lbmap():
    """AddSVC2BPFMap: slaves 1..n carry rev_nat_index = id, the master count = n."""
    topo = RL.topology(DOC)
    sc = RL.compile_case(DOC, CASES[0], topo)
    m = sc.maps["lb4_svc"]
    rows = {bytes(k): bytes(v) for k, v in zip(m.keys, m.vals)}
    vip = bytes([2, 2, 2, 2])
    master = rows[vip + bytes(4)]
    assert int.from_bytes(master[6:8], "little") == 2 and master[8:10] == bytes(2)
    s1 = rows[vip + bytes([0, 0, 1, 0])]
    assert s1[0:4] == RL.addr(DOC, topo, "httpd1", False) and int.from_bytes(s1[8:10], "big") == 1
    assert len(sc.maps["revnat6"].keys) == 2


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_lb_checks(case):
    topo = RL.topology(DOC)
    flows, _ = RL.run_case(DOC, case, topo, RL.OracleBackend(RL.compile_case(DOC, case, topo)))
    bad = RL.mismatches(case, flows)
    assert not bad, bad
    # both backends of a two-backend service take sessions (lb4/6_select_slave by skb hash)
    for check in case["checks"]:
        svc = next(s for s in case["services"] if s["frontend"][0] == check[1])
        if len(svc["backends"]) == 2:
            got = {f.server for f in flows if (f.client, f.target, f.req) == tuple(check[:3])}
            assert len(got) == 2, (check, got)


def test_without_reverse_nat_the_container_pings_fail():
    """Negative control: with the reverse-NAT maps empty the reply reaches the
    client from the backend's address, which ping / curl reject."""
    topo = RL.topology(DOC)
    case = CASES[0]
    sc = RL.compile_case(DOC, case, topo)
    for name in ("revnat4", "revnat6"):
        sc.maps[name].keys = sc.maps[name].vals = None
    flows, _ = RL.run_case(DOC, case, topo, RL.OracleBackend(sc))
    res = RL.outcomes(flows)
    assert not any(res[("client", "2.2.2.2", "ping")]) and not any(res[("client", "f00d::1:1", "ping6")])
    assert all(res[("host", "2.2.2.2", "ping")])            # bpf_lb's path has no reverse NAT to lose


def test_without_services_nothing_reaches_a_backend():
    topo = RL.topology(DOC)
    case = copy.deepcopy(CASES[2])
    sc_case = dict(case, services=[])
    flows, _ = RL.run_case(DOC, case, topo, RL.OracleBackend(RL.compile_case(DOC, sc_case, topo)))
    assert all(not any(v) for v in RL.outcomes(flows).values())


@pytest.mark.gpu
def test_gpu_matches_reference_lb_checks_and_oracle():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    from oracle import parity as PY
    topo = RL.topology(DOC)
    for case in CASES:
        gpu = RL.GpuBackend(RL.compile_case(DOC, case, topo))
        ref = RL.OracleBackend(RL.compile_case(DOC, case, topo))
        try:
            gflows, glog = RL.run_case(DOC, case, topo, gpu)
            oflows, olog = RL.run_case(DOC, case, topo, ref)
            assert not RL.mismatches(case, gflows), (case["name"], RL.mismatches(case, gflows))
            assert [(k, s) for k, s, *_ in glog] == [(k, s) for k, s, *_ in olog], case["name"]
            for (kind, step, g, gs), (_, _, o, os_) in zip(glog, olog):
                bad, first = PY.compare_records(g, o)
                assert bad == 0, (case["name"], kind, step, g[first], o[first])
                assert np.array_equal(gs, os_), (case["name"], kind, step)
            for name, ksz in (("ct4", 14), ("ct6", 40)):
                gk, gv = gpu.dump(name, ksz)
                ok, ov = ref.dp.m[name].dump_arrays()
                n, badc = PY.compare_tables(gk, gv, ok, ov)
                assert badc == 0 and n == len(ok), (case["name"], name, n, badc)
        finally:
            gpu.close()
