"""Benchmark: BASELINE config 2 — bpf_lxc ingress (ct_lookup4 + policy_can_access)
over a steady-state stream of 16M-packet batches (4M new flows per step, each
flow spans 4 steps), 2^20 address pairs, 4,352 identities, 256 endpoints.

One step = gf_policy_ingress_classify over one batch resident in HBM (flow-group
grouping + CT + policy + output).  N GPUs: one process per GPU, flow groups
(unordered address pairs) sharded across ranks, tables replicated, CT
partitioned; the only collective is the RCCL all-reduce of the counter block
(and the timing max).  `python bench.py --gpus N` without a torch.distributed
launcher spawns the N rank processes itself (before anything touches a GPU).

Prints ONE JSON line (rank 0) with roofline, cpu_baseline and parity objects.
`parity` is the full-scale bit-exactness check: the CPU restatement (oracle/)
runs the same stream on a flow-group sample (1/--parity-div of the address
pairs: whole flow groups, so a sampled run of the stateful path is exact) and
every sampled packet's GPU record, plus every CT entry of the sampled pairs at
the end, must equal the oracle's.  At N=1 the line also carries "configs": the
other BASELINE configurations measured the same way (config 1 XDP prefilter,
config 3 service LB, config 4 full pipeline over raw frames, config 5 IPv6
pipeline, and the endpoint egress path of SURVEY §8(f)), each with its own
roofline, CPU baseline and parity (`--config N` prints that configuration
alone as the line).
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpps classified (whole node) + % HBM roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- CPU side facts
def cpu_threads():
    """Threads for the CPU baseline: this process's CPU share (OMP_NUM_THREADS on
    the GPU box, else the affinity mask)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    e = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(int(e), aff)) if e and e.isdigit() else aff


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_base(value, T, sample, single=None):
    return {"value": round(value, 3), "unit": "Mpps", "cores": T, "kind": "port", "cpu_model": cpu_model(),
            "single_core_mpps": None if single is None else round(single, 3), "sample": sample}


# ----------------------------------------------------------------------------- timing
def timed(run_step, W, K, dev, world=1, ranged=False):
    """W untimed warm-up steps, then K steps bracketed by barrier + synchronize,
    with the verdict counter sink and the launch profiler on (ranged: run_step(a, b)
    runs steps a..b-1 in one call).  Returns (elapsed_s (max over ranks), counters
    (summed over ranks), local counters, {kernel: (launches, total_ms)})."""
    import torch
    import torch.distributed as dist
    import ctypes as C
    from cilium_amd._lib import lib, gf_prof_rec
    if ranged:
        run_step(0, W)
    else:
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
    if ranged:
        run_step(W, W + K)
    else:
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
    """Runs fn() (returns packets done) until `seconds` of wall time."""
    done, tt = 0, 0.0
    while tt < seconds:
        a = time.perf_counter()
        done += fn()
        tt += time.perf_counter() - a
    return done, tt


# ----------------------------------------------------------------------------- parity bookkeeping
class Parity:
    """Accumulates the full-scale comparison of one configuration."""

    def __init__(self, sample):
        self.sample, self.packets, self.bad, self.first = sample, 0, 0, None
        self.ct = {}

    def records(self, gpu, ref, where):
        from oracle.parity import compare_records
        bad, first = compare_records(gpu, ref)
        self.packets += len(ref)
        self.bad += bad
        if bad and self.first is None:
            self.first = f"{where} sampled row {first}"

    def table(self, name, gk, gv, rk, rv, gtotal):
        from oracle.parity import compare_tables
        n, bad = compare_tables(gk, gv, rk, rv)
        self.ct[name] = {"entries_compared": n, "mismatches": bad, "gpu_entries_total": int(gtotal)}

    def result(self, steps):
        r = {"packets_compared": int(self.packets), "mismatches": int(self.bad), "steps": steps,
             "sample": self.sample}
        if self.first:
            r["first_mismatch"] = self.first
        if self.ct:
            r["ct_entries_compared"] = int(sum(v["entries_compared"] for v in self.ct.values()))
            r["ct_mismatches"] = int(sum(v["mismatches"] for v in self.ct.values()))
            r["tables"] = self.ct
        return r


def lru_replay(dp, ref):
    """The GPU's LRU evictions (gf_ct_evict_log) replayed by a sampled oracle:
    eviction cutoffs depend on the whole table, which a sample does not hold."""
    import ctypes as C
    from cilium_amd._lib import lib, gf_ct_evict_rec
    for name in ref.lru_maps:
        recs = (gf_ct_evict_rec * 4096)()
        n = lib.gf_ct_evict_log(dp.fd[name], recs, 4096)
        ref.lru_replay[name] = {r.seq: (r.cut_closing, r.cut_other) for r in recs[:max(0, min(n, 4096))]}


def compare_ct(par, dp, ref, name, ksz, div, pred=None):
    from oracle import parity as PY
    pred = pred or PY.ct_sampled
    gk, gv, gtot = PY.gpu_table_sampled(dp.fd[name], ksz, 48, div, pred=pred)
    rk, rv = PY.oracle_table_sampled(ref.m[name], div, pred=pred)
    par.table(name, gk, gv, rk, rv, gtot)


def cols_packets(cdict, idx, v6=False):
    """Host Packets (raw frames) for the rows idx of a column batch."""
    import torch
    from cilium_amd import stream
    from cilium_amd.synth import Packets
    c = {k: v[idx].cpu().numpy() for k, v in cdict.items()}
    to_u = {np.dtype(np.int32): np.uint32, np.dtype(np.int16): np.uint16}
    c = {k: (v.view(to_u[v.dtype]) if v.dtype in to_u else v) for k, v in c.items()}
    f, lens = stream.to_frames6(c) if v6 else stream.to_frames(c)
    return Packets(f, lens, c["src_identity"], c["ifindex"], c["lxc_id"], c["tc_index"])


# ----------------------------------------------------------------------------- config 2 (the headline)
def bench_config2(args, dev, rank, world):
    import torch
    from cilium_amd import synth, stream
    from cilium_amd.datapath import Datapath
    W, K = max(args.warmup, 3), args.steps
    t0 = time.time()
    # Weak scaling: every rank serves --pairs address pairs (its RSS share of
    # pairs x world), so the per-GPU step — packets, flow groups, bucket depth, CT
    # partition — is the N=1 step at every N.
    sc, P, _ = synth.config2_tables(n_pairs=args.pairs * world, ct_max=args.ct_max)
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
    batches, ps = [], []
    for s in range(W + K):
        cols, p, n = st.step(S0 + s)
        batches.append(ColBatch(cols, n, dev))
        ps.append(p)
    # one output buffer per step: the parity leg reads every step's records afterwards
    outs = [torch.empty((b.n, 8), dtype=torch.uint8, device=dev) for b in batches]
    torch.cuda.synchronize()
    log(f"rank {rank}: generated {W + K} steps ({time.time() - t0:.1f}s)")
    now = sc.now
    if not args.pipeline:
        elapsed, c, lc, kern = timed(lambda s: dp.ingress(batches[s], now + s, out=outs[s]), W, K, dev, world)
    else:
        # the stream of batches through gf_policy_ingress_classify_batches: batch s+1's
        # schedule is built on a second stream while handle_policy of batch s runs
        # (measured slower: the overlapped kernels share the memory system)
        elapsed, c, lc, kern = timed(lambda a, b: dp.ingress_batches(batches[a:b], [now + s for s in range(a, b)],
                                                                      outs[a:b]), W, K, dev, world, ranged=True)
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
    cpu = par = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, par = oracle_config2(args, sc, st, dp, batches, ps, outs, W, K)
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
            "address_pairs_per_gpu": int(args.pairs),
            "address_pairs": int(args.pairs) * world,
            "ct_max_entries": int(args.ct_max),
            "ct_entries_at_end": int(bpf_entries(dp, "cilium_ct4_global")),
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
        "parity": par,
    }


def bpf_entries(dp, name):
    from cilium_amd import bpf
    return bpf.GetMapInfo(dp.fd[name]).Entries


class ColBatch:
    """Device columns of one step (dict of tensors) in the DeviceBatch shape."""

    def __init__(self, cols, n, dev):
        from cilium_amd.datapath import DeviceBatch
        self.n, self.device = n, dev
        self.saddr6 = self.daddr6 = self.flow_hash = None
        self.cdict = cols
        for k, v in cols.items():
            setattr(self, k, v)
        self._cols = DeviceBatch.cols

    def cols(self):
        return self._cols(self)


def oracle_config2(args, sc, st, dp, batches, ps, outs, W, K):
    """The CPU restatement (oracle, multi-threaded, RSS-style partition by flow
    group) over the flow-group sample of every step (warm-up included): its
    records must equal the GPU's for every sampled packet and, after the last
    step, its CT must equal the GPU CT's entries of the sampled pairs.  The timed
    steps give the CPU baseline; on the first one, 1/8 of the sampled groups run
    on one core first (exact: flow groups are independent) for the single-core
    figure."""
    import torch
    from cilium_amd.datapath import ING_OUT
    from oracle.scenario import OracleDP
    from oracle import parity as PY
    T, div = cpu_threads(), args.parity_div
    t0 = time.time()
    ref = OracleDP(sc, shards=T)
    lru_replay(dp, ref)
    sa, da = st.p_saddr.cpu().numpy(), st.p_daddr.cpu().numpy()
    samp = torch.from_numpy(PY.pair_sampled(sa, da, div)).to(st.device)
    one = torch.from_numpy(PY.pair_sampled(sa, da, div * 8)).to(st.device)
    par = Parity(f"1/{div} of the address pairs (whole flow groups), every step incl. warm-up")
    done = single_n = 0
    tt = single_t = 0.0
    for s in range(W + K):
        idx = torch.nonzero(samp[ps[s]]).squeeze(1)
        pk = cols_packets(batches[s].cdict, idx)
        gout = outs[s][idx].cpu().numpy().view(ING_OUT).ravel()
        if s == W:
            m1 = one[ps[s]][idx].cpu().numpy()
            a = time.perf_counter()
            r1 = ref.ingress(_sub(pk, np.nonzero(m1)[0]), sc.now + s, threads=1, lru=False)
            single_t = time.perf_counter() - a
            single_n = int(m1.sum())
            a = time.perf_counter()
            r2 = ref.ingress(_sub(pk, np.nonzero(~m1)[0]), sc.now + s, threads=T)
            tt += time.perf_counter() - a
            done += pk.n - single_n
            r = np.empty(pk.n, r1.dtype)
            r[m1], r[~m1] = r1, r2
        else:
            a = time.perf_counter()
            r = ref.ingress(pk, sc.now + s, threads=T)
            if s >= W:
                tt += time.perf_counter() - a
                done += pk.n
        par.records(gout, r, f"step {s}")
    compare_ct(par, dp, ref, "cilium_ct4_global", 14, div)
    log(f"cpu baseline + parity: {par.packets} packets compared, {par.bad} mismatches; CT {par.ct}; "
        f"{done} packets in {tt:.2f}s on {T} threads ({time.time() - t0:.1f}s)")
    cpu = cpu_base(done / tt / 1e6 if tt else 0.0, T,
                   f"{done} packets of the same config-2 stream (flows of 1/{div} of the address pairs, the "
                   f"{K} timed steps after the same {W} warm-up steps), oracle restatement, RSS-style flow-group "
                   f"partition over {T} threads; single core: {single_n} packets of step {W}",
                   single_n / single_t / 1e6 if single_t else None)
    return cpu, par.result(W + K)


def _sub(pk, idx):
    from cilium_amd.synth import Packets
    f = lambda x: None if x is None else np.asarray(x)[idx]
    return Packets(pk.frames[idx], pk.lens[idx], f(pk.src_identity), f(pk.ifindex), f(pk.lxc_id), f(pk.tc_index),
                   f(pk.flow_hash))


# ----------------------------------------------------------------------------- config 1 / 3 (stateless)
def bench_config1(args, dev):
    import torch
    import ctypes as C
    from cilium_amd import synth
    from cilium_amd._lib import lib
    from cilium_amd.datapath import Datapath, DeviceBatch
    sc = synth.config1()
    pk = sc.batches[0]
    dp = Datapath(sc, pin_prefix=None)
    b = DeviceBatch(pk)
    out = torch.empty(b.n, dtype=torch.uint8, device=dev)

    def step(s):
        c = b.cols()
        lib.gf_xdp_classify(dp.xdp_prog, C.byref(c), out.data_ptr(), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    W, K = 5, 50
    el, c, _, kern = timed(step, W, K, dev)
    cpu = par = None
    if not args.no_cpu:
        from oracle.scenario import OracleDP
        from oracle import oracle as O
        T = cpu_threads()
        ref = OracleDP(sc)
        bt = ref.batch(pk)
        r = O.xdp(ref.xdp_cfg, bt, T)
        par = Parity("the whole 1M-packet batch")
        par.records(out.cpu().numpy(), r, "batch")
        done, tt = cpu_loop(lambda: (O.xdp(ref.xdp_cfg, bt, T), pk.n)[1], args.cpu_seconds / 4)
        a = time.perf_counter()
        O.xdp(ref.xdp_cfg, bt, 1)
        t1 = time.perf_counter() - a
        cpu = cpu_base(done / tt / 1e6, T, f"{done} packets (the same 1M-packet batch, repeated)", pk.n / t1 / 1e6)
        par = par.result(1)
    return {"workload": "config1: bpf_xdp CIDR prefilter (10k LPM prefixes + 2k /32, 1025 endpoints), 1M packets/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_xdp"], float(c[270]) / K, "k_xdp"), "kernels_ms_per_step": kms(kern),
            "verdicts": {"pass": int(c[258]), "drop": int(c[257])},
            "cpu_baseline": cpu, "parity": par}


def bench_config3(args, dev):
    import torch
    import ctypes as C
    from cilium_amd import synth
    from cilium_amd._lib import lib
    from cilium_amd.datapath import Datapath, DeviceBatch, LB_OUT
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
    cpu = par = None
    if not args.no_cpu:
        from oracle.scenario import OracleDP
        from oracle import oracle as O
        T = cpu_threads()
        ref = OracleDP(sc)
        bt = ref.batch(pk)
        a = time.perf_counter()
        r, _ = O.lb(ref.lb_cfg, bt, T)
        tfull = time.perf_counter() - a
        par = Parity("the whole 16M-packet batch")
        par.records(out.cpu().numpy().view(LB_OUT).ravel(), r, "batch")
        sub = pk.slice(0, 1_000_000)
        bs = ref.batch(sub)
        a = time.perf_counter()
        O.lb(ref.lb_cfg, bs, 1)
        t1 = time.perf_counter() - a
        cpu = cpu_base(pk.n / tfull / 1e6, T, f"{pk.n} packets (the whole batch, once)", sub.n / t1 / 1e6)
        par = par.result(1)
    return {"workload": "config3: bpf_lb lb4_lookup_service + slave select, 100k services / ~1M backends, "
                        "16M packets/step (Zipf 1.1)",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_lb"], float(c[270]) / K, "k_lb"), "kernels_ms_per_step": kms(kern),
            "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


# ----------------------------------------------------------------------------- config 4 (full pipeline)
class FrameBatch:
    def __init__(self, frames, lens, tc_index, dev, lxc_id=None, flow_hash=None):
        self.frames, self.len, self.tc_index, self.lxc_id, self.flow_hash = frames, lens, tc_index, lxc_id, flow_hash
        self.n, self.device = frames.shape[0], dev


def bench_config4(args, dev):
    import torch
    from cilium_amd import synth, stream
    from cilium_amd.datapath import Datapath
    W, K = 4, max(4, args.steps // 2)
    sc, P, vip = synth.config4_tables(n_pairs=args.pairs, ct_max=args.ct_max)
    st = stream.Stream(P, flows_per_step=args.flows_per_step, device=dev, vip_ip=vip)
    S0 = 3
    rk, rv = st.reply_ct_entries(S0 + W + K)
    sc.maps["cilium_ct4_global"].keys, sc.maps["cilium_ct4_global"].vals = rk, rv
    dp = Datapath(sc, pin_prefix=None)
    fbs, ps = [], []
    for s in range(W + K):
        cols, p, n = st.step(S0 + s)
        f, lens = stream.device_frames(cols)
        fbs.append(FrameBatch(f, lens, cols["tc_index"], dev))
        ps.append(p)
    outs = [torch.empty((b.n, 24), dtype=torch.uint8, device=dev) for b in fbs]
    torch.cuda.synchronize()
    el, c, _, kern = timed(lambda s: dp.pipeline(fbs[s], sc.now + s, out=outs[s], snap_out=False), W, K, dev)
    names = [k for k in kern]
    cpu = par = None
    if not args.no_cpu:
        cpu, par = oracle_config4(args, sc, st, dp, fbs, ps, outs, W, K)
    return {"workload": "config4: bpf_xdp -> bpf_lb -> bpf_netdev delivery -> handle_policy over raw 64-B frames "
                        "(config-2 stream, 30% of pairs via service VIPs; 10k-prefix prefilter), 16.8M packets/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, names, float(c[270]) / K, "all pipeline kernels (frames -> verdicts)"),
            "kernels_ms_per_step": kms(kern), "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


def oracle_config4(args, sc, st, dp, fbs, ps, outs, W, K, ct_names=("cilium_ct4_global",), v6_pairs=None):
    """The oracle pipeline over the flow-group sample of every step (the flow group
    is the post-LB address pair, i.e. the stream's pair), records and the sampled
    pairs' CT entries compared; timed steps give the CPU baseline."""
    import torch
    from cilium_amd.datapath import PIPE_OUT
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    from oracle import parity as PY
    T, div = cpu_threads(), args.parity_div * 2
    ref = OracleDP(sc, shards=T)
    lru_replay(dp, ref)
    if v6_pairs is None:
        sa, da = st.p_saddr.cpu().numpy(), st.p_daddr.cpu().numpy()
        pm = PY.pair_sampled(sa, da, div)
        pm1 = PY.pair_sampled(sa, da, div * 8)
    else:
        pm, pm1 = PY.pair_sampled6(*v6_pairs, div), PY.pair_sampled6(*v6_pairs, div * 8)
    samp, one = torch.from_numpy(pm).to(st.device), torch.from_numpy(pm1).to(st.device)
    par = Parity(f"1/{div} of the address pairs (whole flow groups), every step incl. warm-up")
    done = single_n = 0
    tt = single_t = 0.0
    for s in range(W + K):
        idx = torch.nonzero(samp[ps[s]]).squeeze(1)
        b = fbs[s]
        pk = Packets(b.frames[idx].cpu().numpy(), b.len[idx].cpu().numpy().view(np.uint32),
                     tc_index=None if b.tc_index is None else b.tc_index[idx].cpu().numpy())
        gout = outs[s][idx].cpu().numpy().view(PIPE_OUT).ravel()
        if s == W:
            m1 = one[ps[s]][idx].cpu().numpy()
            a = time.perf_counter()
            r1 = ref.pipeline(_sub(pk, np.nonzero(m1)[0]), sc.now + s, threads=1, lru=False)[0]
            single_t, single_n = time.perf_counter() - a, int(m1.sum())
            a = time.perf_counter()
            r2 = ref.pipeline(_sub(pk, np.nonzero(~m1)[0]), sc.now + s, threads=T)[0]
            tt += time.perf_counter() - a
            done += pk.n - single_n
            r = np.empty(pk.n, r1.dtype)
            r[m1], r[~m1] = r1, r2
        else:
            a = time.perf_counter()
            r = ref.pipeline(pk, sc.now + s, threads=T)[0]
            if s >= W:
                tt += time.perf_counter() - a
                done += pk.n
        par.records(gout, r, f"step {s}")
    for name in ct_names:
        compare_ct(par, dp, ref, name, 14 if "4" in name else 40, div)
    cpu = cpu_base(done / tt / 1e6 if tt else 0.0, T,
                   f"{done} packets (flows of 1/{div} of the address pairs, the {K} timed steps after the same "
                   f"warm-up), {T} threads; single core: {single_n} packets of step {W}",
                   single_n / single_t / 1e6 if single_t else None)
    return cpu, par.result(W + K)


# ----------------------------------------------------------------------------- config 5 (IPv6 pipeline)
def bench_config5(args, dev):
    """BASELINE config 5 through the path an IPv6 packet takes on a node: bpf_xdp's
    check_v6 (v6_dyn LPM, 10k /32-/127 prefixes; v6_fix hash, 100k /128s; endpoint
    check) -> bpf_netdev handle_ipv6 (identity from the flow label of cluster
    sources, hop limit, MACs) -> handle_policy / ipv6_policy with ct_lookup6 on a
    10,485,760-entry LRU CT pre-filled to 8M entries."""
    import torch
    from cilium_amd import synth, stream
    from cilium_amd.datapath import Datapath
    W, K = 3, 4
    t0 = time.time()
    sc, P, meta = synth.config5_tables(n_pairs=args.pairs, prefill=args.ct6_prefill)
    st = stream.Stream6Frames(P, meta, flows_per_step=1 << 20, device=dev)
    S0 = 3
    rk, rv = st.reply_ct6_entries(S0 + W + K)
    ct6 = sc.maps["cilium_ct6_global"]
    ct6.keys, ct6.vals = synth.ct6_prefill(meta, rk, rv, sc.now)
    dp = Datapath(sc, pin_prefix=None)
    log(f"config5: tables + {sc.maps['cilium_ct6_global'].n()} pre-filled CT6 entries ({time.time() - t0:.1f}s)")
    fbs, ps = [], []
    for s in range(W + K):
        f, lens, p = st.step(S0 + s)
        fbs.append(FrameBatch(f, lens, None, dev))
        ps.append(p)
    outs = [torch.empty((b.n, 24), dtype=torch.uint8, device=dev) for b in fbs]
    torch.cuda.synchronize()
    el, c, _, kern = timed(lambda s: dp.pipeline(fbs[s], sc.now + s, out=outs[s], snap_out=False), W, K, dev)
    names = [k for k in kern]
    cpu = par = None
    if not args.no_cpu:
        cpu, par = oracle_config4(args, sc, st, dp, fbs, ps, outs, W, K, ct_names=("cilium_ct6_global",),
                                  v6_pairs=st.pair_addrs6())
    from cilium_amd import bpf
    return {"workload": "config5: IPv6 bpf_xdp check_v6 (10k v6_dyn /32-/127 + 100k v6_fix /128) -> bpf_netdev "
                        "handle_ipv6 -> handle_policy ipv6_policy (ct_lookup6), CT6 max 10,485,760 (LRU) pre-filled "
                        f"to {args.ct6_prefill}, 1M new flows/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "ct6_entries_at_end": int(bpf.GetMapInfo(dp.fd["cilium_ct6_global"]).Entries),
            "ct6_evictions": len(_evictions(dp, "cilium_ct6_global")),
            "roofline": roofline(kern, names, float(c[270]) / K, "all pipeline kernels (frames -> verdicts)"),
            "kernels_ms_per_step": kms(kern), "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


def _evictions(dp, name):
    from cilium_amd._lib import lib, gf_ct_evict_rec
    recs = (gf_ct_evict_rec * 4096)()
    n = lib.gf_ct_evict_log(dp.fd[name], recs, 4096)
    return [(r.seq, r.evicted) for r in recs[:max(0, min(n, 4096))]]


# ----------------------------------------------------------------------------- endpoint egress
def bench_egress(args, dev):
    """The from-container program (handle_ipv4_from_lxc) over frames sent by 256
    local endpoints (synth.TENANT per tenant), local deliveries continuing into handle_policy:
    4M flows, one 64-B frame each per step; each step a quarter of the flows
    starts anew (new source port), the rest are established."""
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
        a = (s % 4) * q                    # a new source port for each flow of this quarter
        sp = base[a:a + q, 34].to(torch.int64) * 256 + base[a:a + q, 35].to(torch.int64)
        sp = 1024 + (sp - 1024 + 7919 * (s + 1)) % 60000
        fs[a:a + q, 34], fs[a:a + q, 35] = (sp >> 8).to(torch.uint8), (sp & 0xff).to(torch.uint8)
        frames.append(fs)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)
    len_t, lid_t, fh_t = t(lens, np.int32), t(lid, np.int16), t(fh, np.int32)
    fbs = [FrameBatch(frames[i], len_t, None, dev, lid_t, fh_t) for i in range(W + K)]
    outs = [torch.empty((n, 24), dtype=torch.uint8, device=dev) for _ in range(W + K)]
    el, c, _, kern = timed(lambda s: dp.egress(fbs[s], sc.now + s, out=outs[s], snap_out=False), W, K, dev)
    log(f"egress: timed {K} steps ({time.time() - t0:.1f}s)")
    cpu = par = None
    if not args.no_cpu:
        cpu, par = oracle_egress(args, sc, meta, dp, frames, lens, lid, fh, outs, W, K)
    return {"workload": "egress: bpf_lxc from-container handle_ipv4_from_lxc (+ handle_policy of local deliveries), "
                        f"256 endpoints, {n} flows/step (35% world, 20% tunnel, 25% local, 20% service "
                        "VIPs), 1/4 new per step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, list(kern), float(c[270]) / K, "all egress kernels (frames -> verdicts)"),
            "kernels_ms_per_step": kms(kern), "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


def oracle_egress(args, sc, meta, dp, frames, lens, lid, fh, outs, W, K):
    """Parity: tenant 0 (a closed set of flow groups: its endpoints only talk to
    each other, their services and remote peers) through the sequential oracle,
    records and CT entries compared.  CPU baseline: T oracle instances side by
    side, one per share of the tenants (flow groups never cross tenants)."""
    import threading
    import torch
    from cilium_amd.datapath import EG_OUT
    from cilium_amd.synth import Packets, TENANT
    from oracle.scenario import OracleDP
    ep_idx = lid.astype(np.int64) - int(meta["lxc_id"][0])
    ten = ep_idx // TENANT
    T = cpu_threads()
    nten = len(meta["ep4"]) // TENANT
    par = Parity(f"tenant 0 of {nten} (its {TENANT} endpoints' flows: a closed set of flow groups), every step"
                 if nten > 1 else "every packet of every step (one tenant)")
    ref = OracleDP(sc)
    lru_replay(dp, ref)
    m0 = np.nonzero(ten == 0)[0]
    m0t = torch.from_numpy(m0).to(frames[0].device)
    for s in range(W + K):
        pk = Packets(frames[s][m0t].cpu().numpy(), lens[m0], None, None, lid[m0], None, fh[m0])
        r, _ = ref.egress(pk, sc.now + s)
        par.records(outs[s][m0t].cpu().numpy().view(EG_OUT).ravel(), r, f"step {s}")
    t0set = {int(x) for x in synth_raw_be(meta["ep4"][:TENANT])}
    pred = lambda k, div: _tenant_keys(k, t0set)
    compare_ct(par, dp, ref, "ct4", 14, 1, pred=pred)
    # CPU baseline: T instances over closed shares of the flow groups, the W + K steps (the
    # timed K measured): a tenant's local and service flows stay together, flows to world
    # and tunnel peers (no translation: the frame's own pair) spread by pair hash
    from oracle import parity as PY
    f0 = frames[0].cpu().numpy()
    dst = f0[:, 30:34].copy().view(">u4").ravel()
    src_raw, dst_raw = f0[:, 26:30].copy().view("<u4").ravel(), f0[:, 30:34].copy().view("<u4").ravel()
    inside = ((dst >> 16) == 0x0a01) | ((dst >> 16) == 0x0a60)          # endpoints 10.1/16, service VIPs 10.96/16
    hsh = (PY._fmix64((np.maximum(src_raw, dst_raw).astype(np.uint64) << np.uint64(32)) |
                      np.minimum(src_raw, dst_raw).astype(np.uint64)) % np.uint64(T)).astype(np.int64)
    owner = np.where(inside, ten % T, hsh)
    shares = [np.nonzero(owner == t)[0] for t in range(T)]
    insts = [OracleDP(sc) for _ in range(T)]
    host_frames = [frames[s].cpu().numpy() for s in range(W + K)]
    tt, done = 0.0, 0
    for s in range(W + K):
        def run(t):
            sh = shares[t]
            insts[t].egress(Packets(host_frames[s][sh], lens[sh], None, None, lid[sh], None, fh[sh]), sc.now + s)
        th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        a = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        if s >= W:
            tt += time.perf_counter() - a
            done += len(lid)
        if tt >= args.cpu_seconds * 2:
            break
    one = OracleDP(sc)
    sh = shares[0][: max(1, len(shares[0]) // 4)]
    a = time.perf_counter()
    one.egress(Packets(host_frames[0][sh], lens[sh], None, None, lid[sh], None, fh[sh]), sc.now)
    t1 = time.perf_counter() - a
    cpu = cpu_base(done / tt / 1e6 if tt else 0.0, T,
                   f"{done} packets (every flow of the timed steps after {W} warm-up steps), {T} oracle instances "
                   f"over tenant shares; single core: {len(sh)} frames of step 0",
                   len(sh) / t1 / 1e6 if t1 else None)
    return cpu, par.result(W + K)


def synth_raw_be(a):
    from cilium_amd.synth import be32_bytes
    return be32_bytes(a).view("<u4").ravel()


def _tenant_keys(keys, t0set):
    w = np.ascontiguousarray(keys[:, :8]).view("<u4")
    return np.isin(w[:, 0], list(t0set)) | np.isin(w[:, 1], list(t0set))


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


# ----------------------------------------------------------------------------- launcher (--gpus N)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n, argv):
    """`bench.py --gpus N` run directly (no torch.distributed launcher): start the N
    rank processes before anything here touches a GPU (each child pins
    LOCAL_RANK), wait for all, return the worst exit status."""
    if not os.environ.get("GPUFLOW_BENCH_SELFTEST"):
        import torch
        vis = torch.cuda.device_count()         # does not initialise the GPU on this image
        if n > vis:
            log(f"--gpus {n} but only {vis} GPU(s) visible")
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def selftest_line(rank, world, backend):
    """The launcher's CPU rehearsal (GPUFLOW_BENCH_SELFTEST=1, gloo): rendezvous,
    the counter-block all-reduce and the single-line output, no GPU."""
    import torch
    import torch.distributed as dist
    c = torch.zeros(512, dtype=torch.int64)
    c[268] = 1000 + rank                      # packets of this rank
    c[133] = rank + 1
    tt = torch.tensor([0.5 + 0.1 * rank], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return {"metric": METRIC, "value": round(int(c[268]) / float(tt.item()) / 1e6, 6), "unit": "Mpps",
            "n_gpus": world, "steps": 1, "warmup": 0, "ms_per_step": round(float(tt.item()) * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "selftest",
            "config": {"workload": "launcher selftest", "backend": backend}, "verdicts": verdicts(c.numpy())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default="2", choices=["1", "2", "3", "4", "5", "egress"],
                    help="BASELINE configuration printed as the line (default: 2, the headline)")
    ap.add_argument("--flows-per-step", type=int, default=4 << 20)
    ap.add_argument("--pairs", type=int, default=1 << 20, help="address pairs per GPU (config 2: x N in total)")
    ap.add_argument("--ct-max", type=int, default=1 << 27,
                    help="CT max_entries (LRU): 134,217,728, above the entries a default run creates")
    ap.add_argument("--ct6-prefill", type=int, default=8_000_000)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and the parity legs")
    ap.add_argument("--pipeline", action="store_true",
                    help="config 2: the steps through gf_policy_ingress_classify_batches (schedule overlap)")
    ap.add_argument("--no-extra", action="store_true", help="config 2 only (skip the other configurations)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--parity-div", type=int, default=4, help="parity sample: 1 in N address pairs")
    ap.add_argument("--egress-flows", type=int, default=4 << 20)
    args = ap.parse_args()

    selftest = bool(os.environ.get("GPUFLOW_BENCH_SELFTEST"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE {world} != --gpus {args.gpus}: the launcher's world size is used")

    import torch
    import torch.distributed as dist
    if selftest:
        if world > 1:
            dist.init_process_group("gloo")
        res = selftest_line(rank, world, "gloo")
        if rank == 0:
            print(json.dumps(res), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
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
               "cpu_baseline": r["cpu_baseline"], "parity": r.get("parity")}
    if rank == 0:
        from cilium_amd import _lib
        res["build_id"] = _lib.BUILD_ID          # gf_build_id(): the sources libgpuflow.so was compiled from
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
