"""Connectivity matrices of the reference's runtime suite (test/runtime/Policies.go
"L3/L4 Checks", "L4Policy Checks", "CIDR" checks; tests/golden/runtime_policies.json)
replayed as packets: the CPU oracle must reproduce every allow/deny the
reference asserts, and the HIP path must produce the oracle's records
bit-for-bit on the same packets.

The older shell tests the verdict names (tests/01-ct.sh, tests/16-cidr-ingress-policy.sh)
exit 0 at their top in this tree — replaced by the Ginkgo suite transcribed
here — so their matrices are not asserted.  01-ct.sh also expects app -> server
traffic to pass under PolicyEnforcement=always without an egress rule, which
1.0's egress enforcement (Policies.go:762-786) contradicts."""
import pytest

from tests import runtime_matrix as RM

DOC = RM.load()
CASES = DOC["cases"]


def _ids():
    return [c["name"] for c in CASES]


def test_fixture_covers_reference_checks():
    assert len(CASES) >= 10
    n = sum(len(RM.expand(c)) for c in CASES)
    assert n >= 80
    assert {c["enforcement"] for c in CASES} == {"default", "always"}
    # both outcomes in both directions of enforcement
    assert any(not ok for c in CASES for *_, ok in RM.expand(c))


def test_agent_restatement_flags():
    """Default enforcement: a direction is enforced only when a rule selecting
    the endpoint has rules in it (GetRulesMatching)."""
    topo = RM.Topology(DOC["endpoints"])
    sc = RM.compile_case(CASES[0], topo)
    fl = {topo.names[i]: c["flags"] for i, c in enumerate(sc.lxc)}
    I, E = RM.S.LXC_POLICY_INGRESS, RM.S.LXC_POLICY_EGRESS
    assert fl["httpd1"] & I and not fl["httpd1"] & E
    assert fl["app3"] & E and not fl["app3"] & I
    assert not fl["app1"] & (I | E)
    sc = RM.compile_case(next(c for c in CASES if c["enforcement"] == "always"), topo)
    assert all(c["flags"] & I and c["flags"] & E for c in sc.lxc)


@pytest.mark.parametrize("case", CASES, ids=_ids())
def test_oracle_matches_reference_matrix(case):
    topo = RM.Topology(RM.case_endpoints(DOC, case))
    res, _ = RM.run_case(case, topo, RM.OracleBackend(RM.compile_case(case, topo)))
    bad = RM.outcome_mismatches(case, res)
    assert not bad, bad


ONE_BATCH = [c for c in CASES if not any(s.startswith("host") for _, s, *_ in c["checks"])]


@pytest.mark.parametrize("case", ONE_BATCH, ids=[c["name"] for c in ONE_BATCH])
def test_oracle_one_batch_request_and_reply(case):
    """Requests, replies and ACKs in one batch: the per-packet order of the
    reference gives the reference's outcomes."""
    topo = RM.Topology(RM.case_endpoints(DOC, case))
    res, _ = RM.run_case_one_batch(case, topo, RM.OracleBackend(RM.compile_case(case, topo)))
    bad = RM.outcome_mismatches(case, res)
    assert not bad, bad


@pytest.mark.gpu
def test_gpu_one_batch_request_and_reply_ordered():
    """The same batches on the HIP path: the ordering check must split them so
    that every record and every CT entry equals the per-packet oracle's."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    from oracle import parity as PY
    for case in ONE_BATCH:
        topo = RM.Topology(RM.case_endpoints(DOC, case))
        gpu = RM.GpuBackend(RM.compile_case(case, topo))
        ref = RM.OracleBackend(RM.compile_case(case, topo))
        try:
            gres, g = RM.run_case_one_batch(case, topo, gpu)
            ores, o = RM.run_case_one_batch(case, topo, ref)
            bad, first = PY.compare_records(g, o)
            assert bad == 0, (case["name"], first, g[first], o[first])
            assert not RM.outcome_mismatches(case, gres), case["name"]
            cts = [(m, 14 if m.startswith("ct4") else 40) for m in ref.dp.m if m.startswith(("ct4", "ct6"))]
            for name, ksz in cts:
                gk, gv = gpu.dump(name, ksz)
                ok, ov = ref.dp.m[name].dump_arrays()
                n, badc = PY.compare_tables(gk, gv, ok, ov)
                assert badc == 0 and n == len(ok), (case["name"], name, n, badc)
        finally:
            gpu.close()


@pytest.mark.gpu
def test_gpu_matches_reference_matrix_and_oracle():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    from oracle import parity as PY
    for case in CASES:
        topo = RM.Topology(RM.case_endpoints(DOC, case))
        sc = RM.compile_case(case, topo)
        gpu = RM.GpuBackend(sc)
        try:
            gres, glog = RM.run_case(case, topo, gpu)
        finally:
            gpu.close()
        ores, olog = RM.run_case(case, topo, RM.OracleBackend(RM.compile_case(case, topo)))
        assert not RM.outcome_mismatches(case, gres), (case["name"], RM.outcome_mismatches(case, gres))
        assert [(k, s) for k, s, _ in glog] == [(k, s) for k, s, _ in olog], case["name"]
        for (kind, step, g), (_, _, o) in zip(glog, olog):
            bad, first = PY.compare_records(g, o)
            assert bad == 0, (case["name"], kind, step, g[first], o[first])


CT_CASES = [c for c in CASES if c["name"].startswith("Conntrack")]


@pytest.mark.parametrize("case", CT_CASES, ids=[c["name"] for c in CT_CASES])
def test_conntrack_case_replies_pass_on_the_ct(case):
    """RuntimeValidatedConntrackTest (connectivity.go:294-478), ConntrackLocal off and
    on (:672-690): the server's replies leave it under PolicyEnforcement=always with no
    egress rule of its own, and enter the client with no ingress rule, only because
    both CT lookups find the request's entries (CT_REPLY on the server's from-container
    lookup and on the client's handle_policy); a new connection the other way (server
    -> client ping) is dropped by the server's egress policy (DROP_POLICY).  With the
    option on, those entries are in the server's and the client's own maps."""
    topo = RM.Topology(RM.case_endpoints(DOC, case))
    be = RM.OracleBackend(RM.compile_case(case, topo))
    res, log = RM.run_case(case, topo, be)
    local = case.get("conntrack_local", [])
    for n in local:
        assert len(be.dp.dump(f"ct4_{n}")) and len(be.dp.dump(f"ct6_{n}")), n
    assert not RM.outcome_mismatches(case, res)
    flows = [RM.Flow(j, c, s, r) for j, (c, s, r, _) in enumerate(RM.expand(case))]
    # wave 1 holds the second packet of every flow that survived wave 0, in flow order
    alive = [f for f, ok in zip(flows, [RM.expected(case)[(f.client, f.server, f.req)] for f in flows]) if ok]
    kind, step, rec = log[1]
    assert kind == "egress" and step == 1 and len(rec) == len(alive)
    for f, r in zip(alive, rec):
        assert r["eg_ct_ret"] == 2 and r["ct_ret"] == 2, (f.client, f.server, f.req, r)   # CT_REPLY both ways
    kind, step, rec = log[0]
    drops = [r for f, r in zip(flows, rec) if f.client == "server"]
    assert drops and all(r["action"] == 2 and r["reason"] == 133 for r in drops)          # DROP_POLICY
