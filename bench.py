"""Benchmark: BASELINE config 2 — bpf_lxc ingress (ct_lookup4 + policy_can_access)
over a steady-state stream of 16M-packet batches (4M new flows per step, each
flow spans 4 steps), 2^20 address pairs, 4,352 identities, 256 endpoints.

One step = gf_policy_ingress_classify over one batch resident in HBM (flow-group
grouping + CT + policy + output).  N GPUs: one process per GPU, flow groups
(unordered address pairs) sharded across ranks, tables replicated, CT
partitioned; the only collective is the RCCL all-reduce of the counter block
(and the timing max).

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects.  At N=1
the line also carries "configs": the other BASELINE configurations measured the
same way (config 1 XDP prefilter, config 3 service LB, config 4 full pipeline
over raw frames, config 5 IPv6 ingress, and the endpoint egress path of SURVEY
§8(f)), each with its own roofline and CPU baseline (`--config N` prints that
configuration alone as the line).
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpps classified (whole node) + % HBM roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- timing
def timed(run_step, W, K, dev, world=1):
    """W untimed warm-up steps, then K steps bracketed by barrier + synchronize,
    with the verdict counter sink and the launch profiler on.  Returns
    (elapsed_s (max over ranks), counters (summed over ranks), local counters,
    {kernel: (launches, total_ms)})."""
    import torch
    import torch.distributed as dist
    import ctypes as C
    from cilium_amd._lib import lib, gf_prof_rec
    for s in range(W):
        run_step(s)
    torch.cuda.synchronize()
    counters = torch.zeros(512, dtype=torch.int64, device=dev)
    lib.gf_set_stats_sink(C.c_void_p(counters.data_ptr()))
    lib.gf_prof_enable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(W, W + K):
        run_step(s)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    lib.gf_set_stats_sink(None)
    recs = (gf_prof_rec * 32)()
    nrec = lib.gf_prof_read(recs, 32)
    lib.gf_prof_enable(0)
    kern = {recs[i].name.decode(): (recs[i].count, recs[i].total_ms) for i in range(nrec)}
    local = counters.clone()
    tt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.all_reduce(counters, op=dist.ReduceOp.SUM)        # RCCL over xGMI: verdict counter block
    return float(tt.item()), counters.cpu().numpy(), local.cpu().numpy(), kern


def roofline(kern, names, ab_per_step, label):
    """achieved = algorithmic bytes per step / the summed average launch time of
    `names` (HIP events on the launch stream)."""
    ms = 0.0
    for n in names:
        c, t = kern.get(n, (0, 0.0))
        ms += t / max(c, 1)
    ach = ab_per_step / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", "kernel": label, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "algorithmic_bytes_per_launch": ab_per_step,
            "avg_launch_ms": round(ms, 4)}


def verdicts(c):
    return {"pass": int(c[256]), "xdp_drop": int(c[257]), "drop": int(c[258]), "redirect": int(c[263]),
            "ct_new": int(c[264]), "ct_established": int(c[265]), "ct_reply": int(c[266]), "ct_related": int(c[267]),
            "drop_reasons": {str(r): int(c[r]) for r in range(1, 256) if c[r]}, "wire_bytes": int(c[269])}


def kms(kern):
    return {k: round(v[1] / max(v[0], 1), 4) for k, v in kern.items()}


def cpu_loop(fn, seconds):
    """Runs fn() (returns packets done) until `seconds` of wall time; Mpps."""
    done, tt = 0, 0.0
    while tt < seconds:
        a = time.perf_counter()
        done += fn()
        tt += time.perf_counter() - a
    return done, tt


# ----------------------------------------------------------------------------- config 2 (the headline)
def bench_config2(args, dev, rank, world):
    import torch
    from cilium_amd import synth, stream
    from cilium_amd.datapath import Datapath
    W, K = max(args.warmup, 3), args.steps
    t0 = time.time()
    sc, P, _ = synth.config2_tables(n_pairs=args.pairs, ct_max=args.ct_max)
    st = stream.Stream(P, rank=rank, world=world, flows_per_step=args.flows_per_step, device=dev)
    # The stream ramps up over its first 3 steps (flows span 4 steps); the run starts at
    # stream step S0 = 3 so that every launch, warm-up included, is a full steady-state
    # batch (the rocprof --stats average over all launches then matches the timed one).
    S0 = 3
    rk, rv = st.reply_ct_entries(S0 + W + K)
    sc.maps["cilium_ct4_global"].keys, sc.maps["cilium_ct4_global"].vals = rk, rv
    log(f"rank {rank}: tables {sum(m.n() for m in sc.maps.values())} entries, {len(rk)} pre-inserted CT, "
        f"{len(st.own)} owned pairs ({time.time() - t0:.1f}s)")
    dp = Datapath(sc, pin_prefix=None)
    batches = [ColBatch(*st.step(S0 + s)[::2], dev) for s in range(W + K)]
    torch.cuda.synchronize()
    log(f"rank {rank}: generated {W + K} steps ({time.time() - t0:.1f}s)")
    out = torch.empty((max(b.n for b in batches), 8), dtype=torch.uint8, device=dev)
    now = sc.now
    elapsed, c, lc, kern = timed(lambda s: dp.ingress(batches[s], now + s, out=out[: batches[s].n]), W, K, dev, world)
    total_pkts = int(c[268])
    local_pkts = sum(batches[s].n for s in range(W, W + K))
    if world == 1 and not os.environ.get("GPUFLOW_DIAG_LIB"):
        assert total_pkts == local_pkts, (total_pkts, local_pkts)
    # roofline of the dominant kernel (k_ing_groups), this rank
    ki = kern.get("k_ing_groups", (0, 0.0))
    avg_ms = ki[1] / max(ki[0], 1)
    ab_per_launch = float(lc[270]) / max(K, 1)
    achieved = ab_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = traffic_src = None
    pmc = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_summary.json")))
    if pmc:
        try:
            j = json.load(open(pmc[-1]))
            if j.get("kernel") == "k_ing_groups" and j.get("traffic_bytes_per_launch"):
                traffic = j["traffic_bytes_per_launch"] * (batches[W].n / float(j["packets_per_launch"]))
                traffic_src = os.path.relpath(pmc[-1], ROOT)
        except Exception:
            traffic = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline_config2(sc, st, W, K, args.cpu_seconds, S0)
    return {
        "metric": METRIC,
        "value": round(total_pkts / elapsed / 1e6, 3),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded config-2 stream generated on device; tables from cilium_amd.synth)",
        "config": {
            "workload": "config2: bpf_lxc ingress handle_policy (ct_lookup4 + policy_can_access), steady-state "
                        "stream, 4M new flows/step (16M active), 256 endpoints, 4352 identities",
            "packets_per_step_per_gpu": int(batches[W].n),
            "address_pairs": int(args.pairs),
            "ct_capacity": int(args.ct_max),
            "parallelism": f"dp{world} (flow-group sharded, tables replicated, CT partitioned)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_ing_groups (CT+policy stage: handle_policy over every packet of the step)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": ab_per_launch,
            "avg_launch_ms": round(avg_ms, 4),
        },
        "kernels_ms_per_step": kms(kern),
        "verdicts": verdicts(c),
        "cpu_baseline": cpu,
    }


class ColBatch:
    """Device columns of one step (dict of tensors) in the DeviceBatch shape."""

    def __init__(self, cols, n, dev):
        from cilium_amd.datapath import DeviceBatch
        self.n, self.device = n, dev
        self.saddr6 = self.daddr6 = self.flow_hash = None
        for k, v in cols.items():
            setattr(self, k, v)
        self._cols = DeviceBatch.cols

    def cols(self):
        return self._cols(self)


def cpu_baseline_config2(sc, st, W, K, seconds, S0):
    """The CPU restatement (oracle, multi-threaded, RSS-style partition by flow
    group) on a bounded sample of the same stream: the flows of half of the
    rank's address pairs, warmed over the same W steps, then timed step by step
    until `seconds` of CPU wall time."""
    from cilium_amd import stream
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    threads = min(16, os.cpu_count() or 1)
    t0 = time.time()
    ref = OracleDP(sc, shards=threads)

    def sample(s):
        cols, p, n = st.step(S0 + s)
        m = (p % 8) < 4
        c = {k: v[m].cpu().numpy() for k, v in cols.items()}
        to_u = {np.dtype(np.int32): np.uint32, np.dtype(np.int16): np.uint16}
        c = {k: (v.view(to_u[v.dtype]) if v.dtype in to_u else v) for k, v in c.items()}
        f, lens = stream.to_frames(c)
        return Packets(f, lens, c["src_identity"], c["ifindex"], c["lxc_id"], c["tc_index"])

    for s in range(W):
        ref.ingress(sample(s), sc.now + s, threads=threads)
    done, tt = 0, 0.0
    for s in range(W, W + K):
        pk = sample(s)
        a = time.perf_counter()
        ref.ingress(pk, sc.now + s, threads=threads)
        tt += time.perf_counter() - a
        done += pk.n
        if tt >= seconds:
            break
    log(f"cpu baseline: {done} packets in {tt:.2f}s on {threads} threads (setup {time.time() - t0:.1f}s)")
    return {"value": round(done / tt / 1e6, 3), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": f"{done} packets of the same config-2 stream (flows of 1/2 of the address pairs, "
                      f"after the same {W} warm-up steps), oracle restatement, RSS-style flow-group partition"}


# ----------------------------------------------------------------------------- config 1 / 3 (stateless)
def bench_config1(args, dev):
    import torch
    from cilium_amd import synth
    from cilium_amd.datapath import Datapath, DeviceBatch
    from oracle.scenario import OracleDP
    sc = synth.config1()
    pk = sc.batches[0]
    dp = Datapath(sc, pin_prefix=None)
    b = DeviceBatch(pk)
    out = torch.empty(b.n, dtype=torch.uint8, device=dev)
    import ctypes as C
    from cilium_amd._lib import lib

    def step(s):
        c = b.cols()
        lib.gf_xdp_classify(dp.xdp_prog, C.byref(c), out.data_ptr(), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    W, K = 5, 50
    el, c, _, kern = timed(step, W, K, dev)
    threads = min(16, os.cpu_count() or 1)
    cpu = None
    if not args.no_cpu:
        ref = OracleDP(sc)
        bt = ref.batch(pk)
        from oracle import oracle as O
        done, tt = cpu_loop(lambda: (O.xdp(ref.xdp_cfg, bt, threads), pk.n)[1], args.cpu_seconds / 4)
        cpu = {"value": round(done / tt / 1e6, 2), "unit": "Mpps", "cores": threads, "kind": "port",
               "sample": f"{done} packets (the same 1M-packet batch, repeated)"}
    return {"workload": "config1: bpf_xdp CIDR prefilter (10k LPM prefixes + 2k /32, 1025 endpoints), 1M packets/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_xdp"], float(c[270]) / K, "k_xdp"), "kernels_ms_per_step": kms(kern),
            "verdicts": {"pass": int(c[258]), "drop": int(c[257])},
            "cpu_baseline": cpu}


def bench_config3(args, dev):
    import torch
    from cilium_amd import synth
    from cilium_amd.datapath import Datapath, DeviceBatch
    from oracle.scenario import OracleDP
    import ctypes as C
    from cilium_amd._lib import lib
    sc = synth.config3(n_packets=16_000_000)
    pk = sc.batches[0]
    dp = Datapath(sc, pin_prefix=None)
    b = DeviceBatch(pk, with_v6=False)
    out = torch.empty((b.n, 12), dtype=torch.uint8, device=dev)

    def step(s):
        c = b.cols()
        lib.gf_lb_classify(dp.lb_prog, C.byref(c), out.data_ptr(), None,
                           C.c_void_p(torch.cuda.current_stream().cuda_stream))
    W, K = 3, 10
    el, c, _, kern = timed(step, W, K, dev)
    threads = min(16, os.cpu_count() or 1)
    cpu = None
    if not args.no_cpu:
        ref = OracleDP(sc)
        sub = pk.slice(0, 2_000_000)
        bt = ref.batch(sub)
        from oracle import oracle as O
        done, tt = cpu_loop(lambda: (O.lb(ref.lb_cfg, bt, threads), sub.n)[1], args.cpu_seconds / 4)
        cpu = {"value": round(done / tt / 1e6, 2), "unit": "Mpps", "cores": threads, "kind": "port",
               "sample": f"{done} packets (the first 2M packets of the batch, repeated)"}
    return {"workload": "config3: bpf_lb lb4_lookup_service + slave select, 100k services / ~1M backends, "
                        "16M packets/step (Zipf 1.1)",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_lb"], float(c[270]) / K, "k_lb"), "kernels_ms_per_step": kms(kern),
            "verdicts": verdicts(c),
            "cpu_baseline": cpu}


# ----------------------------------------------------------------------------- config 4 (full pipeline)
def bench_config4(args, dev):
    import torch
    from cilium_amd import synth, stream
    from cilium_amd.datapath import Datapath
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    W, K = 4, max(4, args.steps // 2)
    sc, P, vip = synth.config4_tables(n_pairs=args.pairs, ct_max=args.ct_max)
    st = stream.Stream(P, flows_per_step=args.flows_per_step, device=dev, vip_ip=vip)
    S0 = 3
    rk, rv = st.reply_ct_entries(S0 + W + K)
    sc.maps["cilium_ct4_global"].keys, sc.maps["cilium_ct4_global"].vals = rk, rv
    dp = Datapath(sc, pin_prefix=None)
    frames = []
    for s in range(W + K):
        cols, p, n = st.step(S0 + s)
        f, lens = stream.device_frames(cols)
        frames.append((f, lens, cols["tc_index"], p))
    torch.cuda.synchronize()

    class FB:
        pass

    def fbatch(i):
        b = FB()
        b.frames, b.len, b.tc_index = frames[i][0], frames[i][1], frames[i][2]
        b.flow_hash, b.n, b.device = None, frames[i][0].shape[0], dev
        return b

    fbs = [fbatch(i) for i in range(W + K)]
    out = torch.empty((max(b.n for b in fbs), 24), dtype=torch.uint8, device=dev)
    el, c, _, kern = timed(lambda s: dp.pipeline(fbs[s], sc.now + s, out=out[: fbs[s].n], snap_out=False),
                           W, K, dev)
    names = [k for k in kern]
    cpu = None if args.no_cpu else cpu_config4(args, sc, frames, W, K)
    return {"workload": "config4: bpf_xdp -> bpf_lb -> bpf_netdev delivery -> handle_policy over raw 64-B frames "
                        "(config-2 stream, 30% of pairs via service VIPs; 10k-prefix prefilter), 16.8M packets/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, names, float(c[270]) / K, "all pipeline kernels (frames -> verdicts)"),
            "kernels_ms_per_step": kms(kern), "verdicts": verdicts(c), "cpu_baseline": cpu}


def cpu_config4(args, sc, frames, W, K):
    """The oracle pipeline on the flows of 1/8 of the address pairs, after the same warm-up."""
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    threads = min(16, os.cpu_count() or 1)
    ref = OracleDP(sc, shards=threads)

    def sample(i):
        m = (frames[i][3] % 8) == 0
        f = frames[i][0][m].cpu().numpy()
        lens = frames[i][1][m].cpu().numpy().view(np.uint32)
        return Packets(f, lens, tc_index=frames[i][2][m].cpu().numpy())

    for s in range(W):
        ref.pipeline(sample(s), sc.now + s, threads=threads)
    done, tt = 0, 0.0
    for s in range(W, W + K):
        pk = sample(s)
        a = time.perf_counter()
        ref.pipeline(pk, sc.now + s, threads=threads)
        tt += time.perf_counter() - a
        done += pk.n
        if tt >= args.cpu_seconds / 2:
            break
    return {"value": round(done / tt / 1e6, 2), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": f"{done} packets (flows of 1/8 of the address pairs, same warm-up)"}


# ----------------------------------------------------------------------------- config 5 (IPv6 ingress)
def bench_config5(args, dev):
    import torch
    from cilium_amd import synth, stream
    from cilium_amd.datapath import Datapath
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    W, K = 3, 4
    ct6_max = 10_485_760
    sc, P, _ = synth.config2_tables(n_pairs=args.pairs, ct_max=1_000_000)
    sc.add_map(synth.MapSpec("cilium_ct6_global", synth.LRU_HASH, 40, 48, ct6_max))
    for e in sc.lxc:
        e["ct6"] = "cilium_ct6_global"
    st = stream.Stream6(P, flows_per_step=1 << 20, device=dev)
    dp = Datapath(sc, pin_prefix=None)
    S0 = 3
    batches = [ColBatch(*st.step(S0 + s)[::2], dev) for s in range(W + K)]
    out = torch.empty((max(b.n for b in batches), 8), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    el, c, _, kern = timed(lambda s: dp.ingress(batches[s], sc.now + s, out=out[: batches[s].n]), W, K, dev)
    cpu = None if args.no_cpu else cpu_config5(sc, st, W, K, S0)
    return {"workload": "config5: bpf_lxc ingress over IPv6 (ct_lookup6 + policy), 1M new flows/step "
                        "(4.2M packets/step), CT capacity 10,485,760 (LRU)",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_ing_groups6", "k_ing_groups"], float(c[270]) / K,
                                 "k_ing_groups<6> (+ <4> for packets without an IPv6 header)"),
            "kernels_ms_per_step": kms(kern), "verdicts": verdicts(c), "cpu_baseline": cpu}


def cpu_config5(sc, st, W, K, S0):
    """The oracle on the IPv6 flows of 1/8 of the address pairs, after the same warm-up."""
    from cilium_amd import stream
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    threads = min(16, os.cpu_count() or 1)
    ref = OracleDP(sc, shards=threads)

    def sample(s):
        cols, p, n = st.step(S0 + s)
        m = (p % 8) == 0
        cc = {k: v[m].cpu().numpy() for k, v in cols.items()}
        to_u = {np.dtype(np.int32): np.uint32, np.dtype(np.int16): np.uint16}
        cc = {k: (v.view(to_u[v.dtype]) if v.dtype in to_u else v) for k, v in cc.items()}
        f, lens = stream.to_frames6(cc)
        return Packets(f, lens, cc["src_identity"], cc["ifindex"], cc["lxc_id"], cc["tc_index"])

    for s in range(W):
        ref.ingress(sample(s), sc.now + s, threads=threads)
    done, tt = 0, 0.0
    for s in range(W, W + K):
        pk = sample(s)
        a = time.perf_counter()
        ref.ingress(pk, sc.now + s, threads=threads)
        tt += time.perf_counter() - a
        done += pk.n
    return {"value": round(done / tt / 1e6, 2), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": f"{done} packets (flows of 1/8 of the address pairs, same warm-up)"}


# ----------------------------------------------------------------------------- endpoint egress
def bench_egress(args, dev):
    """The from-container program (handle_ipv4_from_lxc) over frames sent by 256
    local endpoints, local deliveries continuing into handle_policy: 4M flows,
    one 64-B frame each per step; each step a quarter of the flows starts anew
    (new source port), the rest are established."""
    import torch
    from cilium_amd import synth
    from cilium_amd.datapath import Datapath
    W, K = 3, max(4, args.steps // 2)
    n = args.egress_flows
    t0 = time.time()
    sc, meta = synth.egress_tables(ct_max=args.ct_max)
    f, lens, lid, fh = synth.egress_flows(meta, n)
    dp = Datapath(sc, pin_prefix=None)
    log(f"egress: tables and {n} flows ({time.time() - t0:.1f}s)")
    base = torch.from_numpy(f).to(dev)
    q = n // 4
    frames = []
    for s in range(W + K):
        fs = base.clone()
        a, port = (s % 4) * q, 20000 + 7 * s
        fs[a:a + q, 34], fs[a:a + q, 35] = port >> 8, port & 0xff
        frames.append(fs)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)
    len_t, lid_t, fh_t = t(lens, np.int32), t(lid, np.int16), t(fh, np.int32)

    class FB:
        pass

    def fbatch(i):
        b = FB()
        b.frames, b.len, b.lxc_id, b.flow_hash, b.n, b.device = frames[i], len_t, lid_t, fh_t, n, dev
        return b

    fbs = [fbatch(i) for i in range(W + K)]
    out = torch.empty((n, 24), dtype=torch.uint8, device=dev)
    el, c, _, kern = timed(lambda s: dp.egress(fbs[s], sc.now + s, out=out, snap_out=False), W, K, dev)
    log(f"egress: timed {K} steps ({time.time() - t0:.1f}s)")
    cpu = None
    if not args.no_cpu:
        from oracle.scenario import OracleDP
        from cilium_amd.synth import Packets
        ref = OracleDP(sc)
        m = (lid % 16) == 0
        done, tt = 0, 0.0
        for s in range(W + K):
            pk = Packets(frames[s][torch.from_numpy(m).to(dev)].cpu().numpy(), lens[m], None, None, lid[m], None, fh[m])
            a = time.perf_counter()
            ref.egress(pk, sc.now + s)
            if s >= W:
                tt += time.perf_counter() - a
                done += pk.n
                if tt >= args.cpu_seconds / 2:
                    break
        cpu = {"value": round(done / tt / 1e6, 2), "unit": "Mpps", "cores": 1, "kind": "port",
               "sample": f"{done} packets (the flows of 1/16 of the endpoints, same steps and warm-up), "
                         "sequential oracle restatement"}
    return {"workload": "egress: bpf_lxc from-container handle_ipv4_from_lxc (+ handle_policy of local deliveries), "
                        f"256 endpoints, {n} flows/step (35% world, 20% tunnel, 25% local, 20% service VIPs), "
                        "1/4 new per step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, list(kern), float(c[270]) / K, "all egress kernels (frames -> verdicts)"),
            "kernels_ms_per_step": kms(kern), "verdicts": verdicts(c), "cpu_baseline": cpu}


EXTRA = {"1": bench_config1, "3": bench_config3, "4": bench_config4, "5": bench_config5, "egress": bench_egress}


def add_traffic(cfg, r):
    """roofline.traffic of configuration `cfg` from its committed PMC summary
    (profiles/*pmc_summary_c<cfg>.json: FETCH_SIZE + WRITE_SIZE per launch of the
    roofline kernels, tools/pmc_summary.py), scaled per packet to this run."""
    pmc = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_summary_c{cfg}.json")))
    if not pmc or "roofline" not in r:
        return r
    try:
        j = json.load(open(pmc[-1]))
        ppl = float(j["packets_per_launch"])
        if ppl > 0 and j.get("traffic_bytes_per_launch"):
            r["roofline"]["traffic"] = j["traffic_bytes_per_launch"] * (r["packets_per_step"] / ppl)
            r["roofline"]["traffic_source"] = os.path.relpath(pmc[-1], ROOT)
    except Exception:
        pass
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default="2", choices=["1", "2", "3", "4", "5", "egress"],
                    help="BASELINE configuration printed as the line (default: 2, the headline)")
    ap.add_argument("--flows-per-step", type=int, default=4 << 20)
    ap.add_argument("--pairs", type=int, default=1 << 20)
    ap.add_argument("--ct-max", type=int, default=64_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="config 2 only (skip the other configurations)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--egress-flows", type=int, default=4 << 20)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.config == "2":
        res = bench_config2(args, dev, rank, world)
        if world == 1 and not args.no_extra:
            res["configs"] = {}
            for k, fn in EXTRA.items():
                t0 = time.time()
                try:
                    res["configs"][k] = add_traffic(k, fn(args, dev))
                except Exception as e:                       # reported, never silently dropped
                    res["configs"][k] = {"error": f"{type(e).__name__}: {e}"}
                log(f"config {k}: {res['configs'][k].get('mpps')} Mpps ({time.time() - t0:.1f}s)")
                torch.cuda.empty_cache()
    else:
        if world > 1:
            raise SystemExit("--config other than 2 runs on one GPU")
        r = add_traffic(args.config, EXTRA[args.config](args, dev))
        res = {"metric": METRIC, "value": r["mpps"], "unit": "Mpps", "n_gpus": 1, "steps": r["steps"],
               "warmup": r["warmup"], "ms_per_step": r["ms_per_step"], "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "u32", "data": "synthetic",
               "config": {"workload": r["workload"], "packets_per_step": r["packets_per_step"]},
               "roofline": r["roofline"], "kernels_ms_per_step": r["kernels_ms_per_step"],
               "cpu_baseline": r["cpu_baseline"]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
