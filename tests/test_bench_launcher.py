"""bench.py on N ranks, rehearsed on the CPU (GPUFLOW_BENCH_SELFTEST: gloo ranks,
CPU tensors, small tables, the oracle standing in for the device).  The same
code the GPU run takes: the launcher that spawns the ranks without touching the
HIP runtime, the flow-group-sharded streams, config 4 with frames arriving on
their owner and with the partition + all-to-all exchange, the parity legs on
every rank and their all-reduce, the counter-block all-reduce and the single
JSON line of rank 0."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--pairs", "512", "--flows-per-step", "2048", "--steps", "2", "--warmup", "1", "--ct-max", "65536"]

# The parent runs bench.py's main() in-process and reports whether it imported
# torch (i.e. could have initialised the HIP runtime) before the ranks ended.
_PARENT = r"""
import runpy, sys, json
sys.argv = ["bench.py"] + sys.argv[1:]
rc = 0
try:
    runpy.run_path(%r, run_name="__main__")
except SystemExit as e:
    rc = e.code or 0
print("PARENT " + json.dumps({"rc": rc, "torch_imported": "torch" in sys.modules}), flush=True)
""" % os.path.join(ROOT, "bench.py")


def _run(n, extra=(), visible="0,1"):
    env = dict(os.environ, GPUFLOW_BENCH_SELFTEST="1", HIP_VISIBLE_DEVICES=visible)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-c", _PARENT, "--gpus", str(n)] + SMALL + list(extra), env=env,
                       capture_output=True, text=True, timeout=600, cwd="/tmp")
    parent = json.loads([l for l in p.stdout.splitlines() if l.startswith("PARENT ")][-1][7:])
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return parent, lines, p.stderr


def test_launcher_world_2_rehearsal():
    parent, lines, err = _run(2)
    assert parent == {"rc": 0, "torch_imported": False}, err[-3000:]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 2 and r["scaling"] == "weak" and r["value"] > 0
    # every packet of both ranks' timed steps is in the all-reduced counter block
    v = r["verdicts"]
    assert v["pass"] + v["drop"] + v["redirect"] == 2 * r["config"]["packets_per_step_per_gpu"] * r["steps"]
    # parity on each rank, summed
    p = r["parity"]
    assert p["ranks"] == 2 and p["mismatches"] == 0 and p["ct_mismatches"] == 0
    assert p["packets_compared"] > 10_000 and p["ct_entries_compared"] > 1_000
    c4, c4x = r["configs"]["4"], r["configs"]["4x"]
    for c in (c4, c4x):
        assert c["n_gpus"] == 2 and c["parity"]["mismatches"] == 0 and c["parity"]["ct_mismatches"] == 0
        assert c["parity"]["packets_compared"] > 5_000 and c["parity"]["ranks"] == 2
    assert "all-to-all" in c4x["ingest"] and "owns" in c4["ingest"]
    # the exchange moved every frame to its owner: the same packets, the same verdicts
    assert c4["verdicts"] == c4x["verdicts"] and c4["packets_per_step"] == c4x["packets_per_step"]
    assert c4["parity"]["packets_compared"] == c4x["parity"]["packets_compared"]


def test_launcher_world_8_rehearsal():
    """The node the driver's scaling run uses: 8 ranks (gloo here, RCCL there), each
    with its own flow groups and CT partition, parity on every rank, the counter
    block all-reduced; config 4 owned and re-partitioned (all-to-all over 8 ranks)."""
    parent, lines, err = _run(8, visible="0,1,2,3,4,5,6,7")
    assert parent == {"rc": 0, "torch_imported": False}, err[-3000:]
    r = lines[0]
    assert r["n_gpus"] == 8 and r["value"] > 0
    v = r["verdicts"]
    assert v["pass"] + v["drop"] + v["redirect"] == 8 * r["config"]["packets_per_step_per_gpu"] * r["steps"]
    p = r["parity"]
    assert p["ranks"] == 8 and p["mismatches"] == 0 and p["ct_mismatches"] == 0 and p["ranks_with_mismatch"] == 0
    for k in ("4", "4x"):
        c = r["configs"][k]
        assert c["n_gpus"] == 8 and c["parity"]["ranks"] == 8 and c["parity"]["mismatches"] == 0
        assert c["parity"]["ct_mismatches"] == 0
    assert r["configs"]["4"]["verdicts"] == r["configs"]["4x"]["verdicts"]
    # the line a first 8-GPU run is diagnosed from: every rank's step time, its
    # k_ing_groups average and the counter all-reduce's cost, and what each rank compared
    rk = r["ranks"]
    for k in ("ms_per_step", "k_ing_groups_avg_ms", "counter_allreduce_ms", "packets"):
        assert len(rk[k]["per_rank"]) == 8 and rk[k]["min"] <= rk[k]["max"], (k, rk[k])
    assert rk["packets"]["per_rank"] == [r["config"]["packets_per_step_per_gpu"] * r["steps"]] * 8
    assert abs(rk["ms_per_step"]["max"] - r["ms_per_step"]) <= 1e-3 * r["ms_per_step"] + 1e-3
    assert len(p["packets_compared_per_rank"]) == 8 and sum(p["packets_compared_per_rank"]) == p["packets_compared"]
    assert min(p["packets_compared_per_rank"]) > 0
    for k in ("4", "4x"):
        assert len(r["configs"][k]["ranks"]["ms_per_step"]["per_rank"]) == 8


def test_parity_div_fits_the_host():
    """At N>1 each rank's parity sample is sized to its share of the host's cores."""
    import types
    sys.path.insert(0, ROOT)
    import bench
    a = types.SimpleNamespace(parity_div=0)
    assert bench.parity_div(a, 1, 2, 10 ** 9) == 1                  # N=1: the whole stream
    assert bench.parity_div(a, 8, 16, 201_326_592) == 2             # 16 threads a rank: the floor
    d = bench.parity_div(a, 8, 2, 201_326_592)                      # a 16-core host shared by 8 ranks
    assert d >= 5 and 201_326_592 / d / (2 * bench.ORACLE_MPPS_PER_THREAD * 1e6) <= bench.PARITY_LEG_S
    assert bench.parity_div(types.SimpleNamespace(parity_div=3), 8, 2, 10 ** 9) == 3


def test_launcher_single_rank_and_device_count():
    parent, lines, err = _run(1)
    assert parent["rc"] == 0 and lines[0]["n_gpus"] == 1 and lines[0]["parity"]["mismatches"] == 0, err[-3000:]
    assert lines[0]["configs"]["4"]["parity"]["mismatches"] == 0
    # more ranks than visible GPUs: refused before any rank starts (counted without HIP)
    parent, lines, err = _run(3, visible="0,1")
    assert parent == {"rc": 2, "torch_imported": False} and not lines


def test_visible_gpus_without_hip(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,2")
    assert bench.visible_gpus() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0


def test_egress_sharded_parity_equals_sequential():
    """The egress leg's parity runs T oracle instances over closed flow-group
    shares (bench.oracle_egress).  Rehearsed here with one sequential oracle in
    the device's place, every packet's record and the union of the instances' CT
    tables must equal the sequential run's: the shares really are closed for the
    egress workload (local, service, world and tunnel flows, new flows every step)."""
    env = dict(os.environ, GPUFLOW_BENCH_SELFTEST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "egress", "--egress-flows", "65536",
                        "--steps", "8"], env=env, capture_output=True, text=True, timeout=600, cwd="/tmp")
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    par = r["parity"]
    assert "oracle instances over closed flow-group shares" in par["sample"], par
    assert par["mismatches"] == 0 and par["ct_mismatches"] == 0, par
    assert par["packets_compared"] == 65536 * par["steps"] and par["ct_entries_compared"] > 100_000


def test_config5_independent_eviction_rehearsal():
    """Config 5's parity leg runs the oracle over the whole stream without the
    device's eviction log: its own LRU stand-in picks the cutoffs from its own
    table, and the two logs are compared entry for entry (rehearsed: a small CT6
    that evicts on most steps)."""
    env = dict(os.environ, GPUFLOW_BENCH_SELFTEST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "5", "--pairs", "4096",
                        "--ct6-prefill", "30000", "--ct6-max", "32768", "--c5-flows", "8192"],
                       env=env, capture_output=True, text=True, timeout=600, cwd="/tmp")
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    ev = r["parity"]["evictions"]["cilium_ct6_global"]
    assert ev["evict_log_equal"] and ev["sweeps_device"] >= 3 and ev["entries_evicted"] > 10_000, ev
    assert r["parity"]["mismatches"] == 0 and r["parity"]["ct_mismatches"] == 0


def test_config2_ct_local_rehearsal():
    """bench.py --ct-local (config 2 with every endpoint on a CT map of its own, the
    ConntrackLocal option): the pre-inserted entries split by their endpoint address,
    every map compared with the oracle's and the evictions of every map equal
    (rehearsed with maps small enough to evict)."""
    env = dict(os.environ, GPUFLOW_BENCH_SELFTEST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--ct-local", "--no-extra", "--pairs", "4096",
                        "--flows-per-step", "16384", "--steps", "4", "--warmup", "3", "--long-steps", "12",
                        "--ct-max", "65536"], env=env, capture_output=True, text=True, timeout=600, cwd="/tmp")
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    par = r["parity"]
    (name, t), = par["tables"].items()
    assert name.endswith("per-endpoint maps") and t["mismatches"] == 0 and t["entries_compared"] > 10_000, par
    (_, ev), = par["evictions"].items()
    assert ev["evict_log_equal"] and ev["sweeps_device"] > 0, ev
    assert par["mismatches"] == 0 and "ConntrackLocal" in r["config"]["workload"]


def test_egress_ct_local_sharded_parity_rehearsal():
    """The egress leg with every endpoint on CT maps of its own: the oracle instances'
    shares stay closed per map (a map's entries come from its endpoint's own sends and
    deliveries), so the union of their copies of each map equals the sequential run's."""
    env = dict(os.environ, GPUFLOW_BENCH_SELFTEST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "egress", "--ct-local",
                        "--egress-flows", "65536", "--steps", "8"], env=env, capture_output=True, text=True,
                       timeout=600, cwd="/tmp")
    r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    par = r["parity"]
    (name, t), = par["tables"].items()
    assert name == "256 per-endpoint maps" and t["mismatches"] == 0 and t["entries_compared"] > 100_000, par
    assert par["mismatches"] == 0 and par["packets_compared"] == 65536 * par["steps"]
