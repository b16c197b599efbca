"""The measurement model behind the bench line's bounds (host logic, no GPU):
tools/pmc_kernels.py turns rocprofv3 --pmc CSVs into per-kernel bytes with the
gfx950 request-size correction (a 128-B read request is 128 B, not the 64 B
FETCH_SIZE prices it at), per-kind request counts and the L2 hit rate; bench.py's
add_bounds uses such a summary only when it was built from the loaded library."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PK = 1000          # packets per step of the synthetic run
STEPS = 4          # warm-up + timed steps the pass ran


def _write_pass(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _summary(tmp_path, build_id="abc"):
    """Two passes over one run: k_ing_pack (the step's first kernel) then k_ing_groups,
    STEPS dispatches each; per dispatch of k_ing_groups 3000 read requests (2500 of
    them 128 B, 100 of 32 B), 2500 write requests (1000 of 64 B, 300 atomics), 700 L2
    hits and 300 misses."""
    p1, p2 = [], []
    for s in range(STEPS):
        pack, groups = 2 * s, 2 * s + 1
        p1 += [{"Dispatch_Id": pack, "Kernel_Name": "k_ing_pack(gf_pkt_cols)", "Counter_Name": "TCC_EA0_RDREQ_sum",
                "Counter_Value": 10}]
        for n, v in (("TCC_EA0_RDREQ_sum", 3000), ("TCC_EA0_RDREQ_32B_sum", 100), ("TCC_EA0_RDREQ_128B_sum", 2500),
                     ("TCC_EA0_WRREQ_sum", 2500)):
            p1.append({"Dispatch_Id": groups, "Kernel_Name": "void k_ing_groups<4>(IngCtx)", "Counter_Name": n,
                       "Counter_Value": v})
        for n, v in (("TCC_EA0_WRREQ_64B_sum", 1000), ("TCC_EA0_ATOMIC_sum", 300), ("TCC_HIT_sum", 700),
                     ("TCC_MISS_sum", 300)):
            p2.append({"Dispatch_Id": groups, "Kernel_Name": "void k_ing_groups<4>(IngCtx)", "Counter_Name": n,
                       "Counter_Value": v})
    _write_pass(str(tmp_path / "pmc" / "p1"), p1)
    _write_pass(str(tmp_path / "pmc" / "p2"), p2)
    bj = tmp_path / "p1.json"
    bj.write_text(json.dumps({"steps": STEPS - 1, "warmup": 1, "packets_per_step": PK, "build_id": build_id}) + "\n")
    out = tmp_path / "summary.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_kernels.py"), str(tmp_path / "pmc"),
                    "--bench-json", str(bj), "--out", str(out)], check=True, capture_output=True)
    return json.load(open(out))


def test_corrected_bytes_and_request_kinds(tmp_path):
    s = _summary(tmp_path)
    k = s["kernels"]["k_ing_groups"]
    assert s["packets_per_step"] == PK and s["steps_run"] == STEPS
    assert k["dispatches_per_step"] == 1.0
    # reads: 128 B x 2500 + 32 B x 100 + 64 B x the other 400; writes: 64 B x 1000 + 32 B x 1500
    assert k["read_bytes"] == 128 * 2500 + 32 * 100 + 64 * 400
    assert k["write_bytes"] == 64 * 1000 + 32 * 1500
    assert k["traffic_bytes_per_packet"] == pytest.approx((k["read_bytes"] + k["write_bytes"]) / PK)
    pp = k["per_packet"]
    assert pp == {"line_reads": 3.0, "reads_128B": 2.5, "partial_writes": 1.2, "full_writes_64B": 1.0, "atomics": 0.3}
    assert k["l2_hit_rate"] == 0.7
    assert k["ea_requests_per_packet"] == pytest.approx(5.5)


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_add_bounds_uses_only_a_summary_of_the_loaded_build(tmp_path, monkeypatch):
    from cilium_amd import _lib
    bench = _bench()
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    path = tmp_path / "profiles" / f"{bench.PMC_ROUND}_pmc_kernels_c2.json"

    def line():
        return {"roofline": {"avg_launch_ms": 0.0002}, "packets_per_step": PK}

    r = bench.add_bounds("2", line())                              # no summary at all
    assert r["roofline"]["bounds_source"].startswith("missing")
    path.write_text(json.dumps(_summary(tmp_path / "a", build_id="not-this-build")))
    r = bench.add_bounds("2", line())                              # another build's summary: stale, unused
    assert r["roofline"]["bounds_stale"]["library_build_id"] == _lib.BUILD_ID
    assert "traffic" not in r["roofline"] and "memory" not in r["roofline"]
    path.write_text(json.dumps(_summary(tmp_path / "b", build_id=_lib.BUILD_ID)))
    rf = bench.add_bounds("2", line())["roofline"]
    assert "bounds_error" not in rf
    assert rf["traffic"] == pytest.approx((128 * 2500 + 32 * 100 + 64 * 400 + 64 * 1000 + 32 * 1500))
    assert rf["l2_hit_rate"] == 0.7
    m = rf["memory"]
    # 1.2 partial writes per packet x 1000 packets in 0.2 us = 6e12/s against 21.7 G/s
    assert m["kinds"]["partial_writes"]["frac"] == pytest.approx(1.2 * PK / 2e-7 / 21.7e9, rel=1e-3)
    assert m["binding"] == max(m["kinds"], key=lambda n: m["kinds"][n]["frac"])
