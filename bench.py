"""Benchmark: BASELINE config 2 — bpf_lxc ingress (ct_lookup4 + policy_can_access)
over a steady-state stream of 16M-packet batches (4M new flows per step, each
flow spans 4 steps), 2^20 address pairs, 4,352 identities, 256 endpoints.

One step = gf_policy_ingress_classify over one batch resident in HBM (flow-group
grouping + CT + policy + output).  N GPUs: one process per GPU, flow groups
(unordered address pairs) sharded across ranks, tables replicated, CT
partitioned; the only collective on the classify path is the RCCL all-reduce of
the counter block (and the timing max).  `python bench.py --gpus N` without a
torch.distributed launcher spawns the N rank processes itself, before anything
in this process touches the HIP runtime.

Prints ONE JSON line (rank 0) with roofline, cpu_baseline and parity objects.
`parity` is the full-scale bit-exactness check: the CPU restatement (oracle/)
runs the same stream on a flow-group sample (1/--parity-div of the address
pairs: whole flow groups, so a sampled run of the stateful path is exact) and
every sampled packet's GPU record, plus every CT entry of the sampled pairs at
the end, must equal the oracle's.  Every rank checks its own partition and the
counts are summed over ranks.  The line also carries "configs": at N=1 the other
BASELINE configurations measured the same way (config 1 XDP prefilter, config 3
service LB, config 4 full pipeline over raw frames — device-resident and with
the host->device copy of the frames —, config 5 IPv6 pipeline, and the endpoint
egress path of SURVEY §8(f)); at N>1 config 4 across the ranks, with frames
arriving on their owner rank (RSS-style) and with frames arriving anywhere and
re-partitioned by gf_pipeline_partition + one all-to-all (`--config N` prints
that configuration alone as the line).

GPUFLOW_BENCH_SELFTEST=1 runs the same code on the CPU (gloo ranks, CPU tensors,
small tables) with the oracle standing in for the device: a rehearsal of the
launcher, the rank / stream / parity / all-reduce logic — it measures nothing.
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
def cpu_threads(local_world=1):
    """Threads for the CPU legs of one rank: this process's CPU share
    (OMP_NUM_THREADS on the GPU box, else the affinity mask), split between the
    node's local ranks."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    e = os.environ.get("OMP_NUM_THREADS")
    t = max(1, min(int(e), aff)) if e and e.isdigit() else aff
    return max(1, min(t, aff // max(1, local_world)))


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


# ----------------------------------------------------------------------------- backends
class Gpu:
    """The product path: libgpuflow's kernels on this rank's GPU (HIP streams,
    the launch profiler and the device counter block)."""
    rehearsal = False
    tables_kw = {}
    ct_max_cap = None

    def __init__(self, local):
        import torch
        # GPUFLOW_BENCH_SHARE_GPU: several ranks on one device (a rehearsal of the
        # N-rank path on a one-GPU box, with GPUFLOW_BENCH_BACKEND=gloo)
        if os.environ.get("GPUFLOW_BENCH_SHARE_GPU"):
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)

    @staticmethod
    def close(dp):
        """Release a datapath's device tables (the next configuration's need the HBM)."""
        dp.close()

    def sync(self):
        import torch
        torch.cuda.synchronize()

    def datapath(self, sc):
        from cilium_amd.datapath import Datapath
        return Datapath(sc, pin_prefix=None)

    def begin(self):
        """Counter sink + launch profiler on (the timed region)."""
        import torch
        import ctypes as C
        from cilium_amd._lib import lib
        self.c = torch.zeros(512, dtype=torch.int64, device=self.dev)
        lib.gf_set_stats_sink(C.c_void_p(self.c.data_ptr()))
        lib.gf_prof_enable(1)
        if hasattr(lib, "gf_diag_wrstats"):              # GF_WRSTATS diagnostic builds only
            lib.gf_diag_wrstats((C.c_ulonglong * 16)(), 16)

    def end(self):
        """(counter block, {kernel: (launches, total_ms)}) of the timed region."""
        from cilium_amd._lib import lib, gf_prof_rec
        lib.gf_set_stats_sink(None)
        recs = (gf_prof_rec * 32)()
        nrec = lib.gf_prof_read(recs, 32)
        lib.gf_prof_enable(0)
        self.wr = None
        if hasattr(lib, "gf_diag_wrstats"):
            import ctypes as C
            v = (C.c_ulonglong * 16)()
            lib.gf_diag_wrstats(v, 16)
            names = ["out", "hit_hot", "carry", "claim_cas", "slot_header", "slot_hot", "side_cold", "related_hot",
                     "related_full", "related_new", "delete", "policy_counter_atomics", "related_log", "strict_count"]
            self.wr = {n: int(v[k]) for k, n in enumerate(names)}
        return self.c, {recs[i].name.decode(): (recs[i].count, recs[i].total_ms) for i in range(nrec)}

    def evict_log(self, dp, name):
        from cilium_amd._lib import lib, gf_ct_evict_rec
        recs = (gf_ct_evict_rec * 4096)()
        n = lib.gf_ct_evict_log(dp.fd[name], recs, 4096)
        return [(r.seq, r.now_sec, r.age_cut, r.hand_line, r.lines, r.evicted) for r in recs[:max(0, min(n, 4096))]]

    def table_sampled(self, dp, name, ksz, div, pred):
        from oracle import parity as PY
        return PY.gpu_table_sampled(dp.fd[name], ksz, 48, div, pred=pred)

    def entries(self, dp, name):
        from cilium_amd import bpf
        return bpf.GetMapInfo(dp.fd[name]).Entries

    def partition(self, dp, fb, rank, world):
        from cilium_amd import shard
        return shard.partition(dp, fb.frames, fb.len, rank, world, fb.flow_hash, fb.tc_index)


class Rehearsal:
    """GPUFLOW_BENCH_SELFTEST: the bench's rank / stream / parity / all-reduce code
    on the CPU (gloo, CPU tensors, small tables) with the oracle standing in for
    the device.  It checks the harness, never the kernels: its numbers are not
    measurements."""
    rehearsal = True
    tables_kw = {"n_ep": 16, "n_ids": 256, "n_l3": 64, "n_l4": 128, "n_wc": 8, "n_cidr": 16}
    ct_max_cap = 1 << 20

    def __init__(self):
        import torch
        self.dev = torch.device("cpu")
        self.c = None

    def sync(self):
        pass

    def datapath(self, sc):
        return StandIn(sc, self)

    @staticmethod
    def close(dp):
        pass

    def begin(self):
        import torch
        self.c = torch.zeros(512, dtype=torch.int64)

    def end(self):
        c, self.c = self.c, None
        return c, {}

    def count(self, rec, lens):
        """The counter block's bins from the stand-in's records (reason, action,
        CT result, packets, wire bytes)."""
        if self.c is None:
            return
        import torch
        h = np.zeros(512, np.int64)
        h[:256] += np.bincount(rec["reason"], minlength=256)[:256]
        h[256:264] += np.bincount(rec["action"], minlength=8)[:8]
        h[264:268] += np.bincount(np.minimum(rec["ct_ret"], 3), minlength=4)[:4]
        h[268] += len(rec)
        h[269] += int(np.asarray(lens, np.int64).sum())
        self.c += torch.from_numpy(h)

    def evict_log(self, dp, name):
        return list(dp.ref.lru_log.get(name, []))

    def table_sampled(self, dp, name, ksz, div, pred):
        from oracle import parity as PY
        k, v = PY.oracle_table_sampled(dp.ref.m[name], div, pred=pred)
        return k, v, dp.ref.m[name].count()

    def entries(self, dp, name):
        return dp.ref.m[name].count()

    def partition(self, dp, fb, rank, world):
        import torch
        from cilium_amd.synth import Packets
        from oracle.parity import owners_host
        pk = Packets(fb.frames.numpy(), fb.len.numpy().view(np.uint32),
                     tc_index=None if fb.tc_index is None else fb.tc_index.numpy())
        lo, nd6 = dp.ref.lb(pk)
        own = owners_host(lo, nd6, pk, rank, world)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int32))
        return t(own), t(np.argsort(own, kind="stable")), t(np.bincount(own, minlength=world))


class StandIn:
    """The oracle in the device's place (Rehearsal only): the classify calls of
    cilium_amd.datapath.Datapath over CPU tensors."""

    def __init__(self, sc, be):
        from oracle.scenario import OracleDP
        self.sc, self.be, self.ref = sc, be, OracleDP(sc)

    def _put(self, out, r):
        import torch
        out.copy_(torch.from_numpy(np.ascontiguousarray(r).view(np.uint8).reshape(len(r), -1)))

    def ingress(self, b, now, out):
        import torch
        pk = cols_packets(b.cdict, torch.arange(b.n))
        r = self.ref.ingress(pk, now)
        self._put(out, r)
        self.be.count(r, pk.lens)
        return out

    def ingress_batches(self, bs, nows, outs):
        return [self.ingress(b, n, o) for b, n, o in zip(bs, nows, outs)]

    def pipeline(self, fb, now, out, snap_out=False):
        from cilium_amd.synth import Packets
        pk = Packets(fb.frames.numpy(), fb.len.numpy().view(np.uint32),
                     tc_index=None if fb.tc_index is None else fb.tc_index.numpy())
        r, _, rs = self.ref.pipeline(pk, now)
        self._put(out, r)
        self.be.count(r, pk.lens)
        import torch
        return out, None, torch.from_numpy(np.ascontiguousarray(rs)) if snap_out else None

    def egress(self, fb, now, out, snap_out=False):
        from cilium_amd.synth import Packets
        pk = Packets(fb.frames.numpy(), fb.len.numpy().view(np.uint32), None, None,
                     fb.lxc_id.numpy().view(np.uint16), None, fb.flow_hash.numpy().view(np.uint32))
        r, _ = self.ref.egress(pk, now)
        self._put(out, r)
        self.be.count(r, pk.lens)
        return out


# ----------------------------------------------------------------------------- timing
def timed(B, run_step, W, K, world=1, ranged=False):
    """W untimed warm-up steps, then K steps bracketed by barrier + synchronize,
    with the verdict counter sink and the launch profiler on (ranged: run_step(a, b)
    runs steps a..b-1 in one call).  Returns (elapsed_s (max over ranks), counters
    (summed over ranks), local counters, {kernel: (launches, total_ms)})."""
    import torch
    import torch.distributed as dist
    if ranged:
        run_step(0, W)
    else:
        for s in range(W):
            run_step(s)
    B.sync()
    B.begin()
    if world > 1:
        dist.barrier()
    B.sync()
    t0 = time.perf_counter()
    host = 0.0                                          # time inside the calls (host enqueue work + waits)
    if ranged:
        run_step(W, W + K)
    else:
        for s in range(W, W + K):
            h0 = time.perf_counter()
            run_step(s)
            host += time.perf_counter() - h0
    B.sync()
    t1 = time.perf_counter()
    if not ranged:
        log(f"host time inside the classify calls: {host / K * 1e3:.3f} ms/step of {(t1 - t0) / K * 1e3:.3f}")
    if world > 1:
        dist.barrier()
    counters, kern = B.end()
    local = counters.clone()
    B.local_elapsed = t1 - t0
    tt = torch.tensor([t1 - t0], dtype=torch.float64, device=B.dev)
    B.allreduce_ms = None
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        B.sync()
        a = time.perf_counter()
        dist.all_reduce(counters, op=dist.ReduceOp.SUM)        # RCCL over xGMI: verdict counter block
        B.sync()
        B.allreduce_ms = (time.perf_counter() - a) * 1e3
    return float(tt.item()), counters.cpu().numpy(), local.cpu().numpy(), kern


def rank_diag(B, world, vals):
    """Each rank's figures side by side (one all_gather): {name: [rank 0, ..]}
    plus min / max, so an N>1 line shows which rank set the max-over-ranks time."""
    import torch
    import torch.distributed as dist
    names = list(vals)
    t = torch.tensor([float(vals[k] if vals[k] is not None else float("nan")) for k in names], dtype=torch.float64,
                     device=B.dev)
    g = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(g, t)
    rows = [x.cpu().tolist() for x in g]
    out = {}
    for i, k in enumerate(names):
        col = [round(r[i], 4) for r in rows]
        out[k] = {"per_rank": col, "min": min(col), "max": max(col)}
    return out


def roofline(kern, names, ab_per_step, label, steps):
    """achieved = algorithmic bytes per step / the device time per step of `names`
    (HIP events on the launch stream around each launch scope, summed over the
    timed steps and divided by their number: a scope launched twice per step
    counts twice)."""
    ms = 0.0
    for n in names:
        c, t = kern.get(n, (0, 0.0))
        ms += t / max(steps, 1)
    ach = ab_per_step / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", "kernel": label, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "frac_source": "HIP events on the launch stream (this run)",
            "traffic": None, "algorithmic_bytes_per_launch": ab_per_step, "avg_launch_ms": round(ms, 4)}


def verdicts(c):
    return {"pass": int(c[256]), "xdp_drop": int(c[257]), "drop": int(c[258]), "redirect": int(c[263]),
            "ct_new": int(c[264]), "ct_established": int(c[265]), "ct_reply": int(c[266]), "ct_related": int(c[267]),
            "drop_reasons": {str(r): int(c[r]) for r in range(1, 256) if c[r]}, "wire_bytes": int(c[269])}


def peak_rss_gb():
    """This process's peak resident set (VmHWM), GB; None where /proc is absent."""
    try:
        for line in open("/proc/self/status"):
            if line.startswith("VmHWM:"):
                return int(line.split()[1]) * 1024 / 1e9
    except OSError:
        pass
    return None


def kms(kern, steps):
    """Device time per step of each launch scope (its launches' summed HIP-event time
    over the timed steps)."""
    return {k: round(v[1] / max(steps, 1), 4) for k, v in kern.items()}


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
    """Accumulates the full-scale comparison of one configuration (one rank)."""

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


def reduce_parity(B, par, rank, world):
    """Parity counts summed over ranks (every rank checked its own flow groups);
    the per-table detail is rank 0's."""
    if world == 1 or par is None:
        return par
    import torch
    import torch.distributed as dist
    t = torch.tensor([par["packets_compared"], par["mismatches"], par.get("ct_entries_compared", 0),
                      par.get("ct_mismatches", 0), 1 if par.get("first_mismatch") else 0], dtype=torch.int64,
                     device=B.dev)
    g = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(g, t)
    per = [x.cpu().tolist() for x in g]
    v = [sum(p[i] for p in per) for i in range(5)]
    r = dict(par)
    r.update({"packets_compared": v[0], "mismatches": v[1], "ct_entries_compared": v[2], "ct_mismatches": v[3],
              "ranks": world, "ranks_with_mismatch": v[4],
              "packets_compared_per_rank": [p[0] for p in per], "ct_entries_compared_per_rank": [p[2] for p in per],
              "sample": par["sample"] + f", on each of the {world} ranks (its own flow groups and CT partition)"})
    if "tables" in r:
        r["tables_rank0"] = r.pop("tables")
    return r


def lru_replay(B, dp, ref):
    """The device's LRU evictions (gf_ct_evict_log) replayed by a sampled oracle:
    eviction cutoffs depend on the whole table, which a sample does not hold."""
    for name in ref.lru_maps:
        ref.lru_replay[name] = {e[0]: (e[2], e[3], e[4]) for e in B.evict_log(dp, name)}


def compare_ct(B, par, dp, ref, name, ksz, div, pred=None):
    from oracle import parity as PY
    pred = pred or PY.ct_sampled
    gk, gv, gtot = B.table_sampled(dp, name, ksz, div, pred)
    rk, rv = PY.oracle_table_sampled(ref.m[name], div, pred=pred)
    par.table(name, gk, gv, rk, rv, gtot)


def cols_packets(cdict, idx, v6=False):
    """Host Packets (raw frames) for the rows idx of a column batch (idx None: all).
    IPv4 frames are built on the device (stream.device_frames with TTL 0, byte for
    byte stream.to_frames) and copied once."""
    from cilium_amd import stream
    from cilium_amd.synth import Packets
    if not v6 and cdict["len"].is_cuda:
        sub = cdict if idx is None else {k: v[idx] for k, v in cdict.items()}
        f, lens = stream.device_frames(sub, ttl=0)
        h = {k: sub[k].cpu().numpy() for k in ("src_identity", "ifindex", "lxc_id", "tc_index")}
        to_u = {np.dtype(np.int32): np.uint32, np.dtype(np.int16): np.uint16}
        h = {k: (v.view(to_u[v.dtype]) if v.dtype in to_u else v) for k, v in h.items()}
        return Packets(f.cpu().numpy(), lens.cpu().numpy().view(np.uint32), h["src_identity"], h["ifindex"],
                       h["lxc_id"], h["tc_index"])
    if idx is None:
        idx = slice(None)
    c = {k: v[idx].cpu().numpy() for k, v in cdict.items()}
    to_u = {np.dtype(np.int32): np.uint32, np.dtype(np.int16): np.uint16}
    c = {k: (v.view(to_u[v.dtype]) if v.dtype in to_u else v) for k, v in c.items()}
    f, lens = stream.to_frames6(c) if v6 else stream.to_frames(c)
    return Packets(f, lens, c["src_identity"], c["ifindex"], c["lxc_id"], c["tc_index"])


def _sub(pk, idx):
    from cilium_amd.synth import Packets
    f = lambda x: None if x is None else np.asarray(x)[idx]
    return Packets(pk.frames[idx], pk.lens[idx], f(pk.src_identity), f(pk.ifindex), f(pk.lxc_id), f(pk.tc_index),
                   f(pk.flow_hash))


# ----------------------------------------------------------------------------- config 2 (the headline)
def bench_config2(args, B, rank, world, local_world=1):
    import torch
    from cilium_amd import synth, stream
    W, K = max(args.warmup, 3), args.steps
    t0 = time.time()
    ct_max = min(args.ct_max, B.ct_max_cap or args.ct_max)
    # Weak scaling: every rank serves --pairs address pairs (its RSS share of
    # pairs x world), so the per-GPU step — packets, flow groups, bucket depth, CT
    # partition — is the N=1 step at every N.
    sc, P, _ = synth.config2_tables(n_pairs=args.pairs * world, ct_max=ct_max, **B.tables_kw)
    st = stream.Stream(P, rank=rank, world=world, flows_per_step=args.flows_per_step, device=B.dev)
    # The stream ramps up over its first 3 steps (flows span 4 steps); the run starts at
    # stream step S0 = 3 so that every launch, warm-up included, is a full steady-state
    # batch (the rocprof --stats average over all launches then matches the timed one).
    S0 = 3
    # the long-horizon continuation (N = 1): steps W + K .. L - 1 run after the headline's
    # timed steps on the same datapath, timed on their own, into the LRU sweeps a node
    # reaches once its CT holds max_entries (not with --pipeline: the continuation
    # runs through dp.ingress only, so the steps the device ran are exactly W + K)
    L = max(args.long_steps, W + K) if world == 1 and not args.pipeline else W + K
    rk, rv = st.reply_ct_entries(S0 + L)
    sc.maps["cilium_ct4_global"].keys, sc.maps["cilium_ct4_global"].vals = rk, rv
    ct_names = ct_local_split(sc, P, ct_max) if args.ct_local else ["cilium_ct4_global"]
    log(f"rank {rank}: tables {sum(m.n() for m in sc.maps.values())} entries, {len(rk)} pre-inserted CT, "
        f"{len(st.own)} owned pairs ({time.time() - t0:.1f}s)")
    dp = B.datapath(sc)
    batches, ps = [], []
    for s in range(L):
        cols, p, n = st.step(S0 + s)
        batches.append(ColBatch(cols, n, B.dev))
        ps.append(p)
    # one output buffer per step: the parity leg reads every step's records afterwards
    outs = [torch.empty((b.n, 8), dtype=torch.uint8, device=B.dev) for b in batches]
    B.sync()
    log(f"rank {rank}: generated {L} steps ({time.time() - t0:.1f}s)")
    now = sc.now
    if not args.pipeline:
        elapsed, c, lc, kern = timed(B, lambda s: dp.ingress(batches[s], now + s, out=outs[s]), W, K, world)
    else:
        # the stream of batches through gf_policy_ingress_classify_batches: batch s+1's
        # schedule is built on a second stream while handle_policy of batch s runs
        # (measured slower: the overlapped kernels share the memory system)
        elapsed, c, lc, kern = timed(B, lambda a, b: dp.ingress_batches(batches[a:b], [now + s for s in range(a, b)],
                                                                         outs[a:b]), W, K, world, ranged=True)
    total_pkts = int(c[268])
    wr = getattr(B, "wr", None)                          # GF_WRSTATS builds: writes by source, timed steps
    long_h = None
    if L > W + K:
        C_ = L - W - K
        el2, c2, _, kern2 = timed(B, lambda s: dp.ingress(batches[W + K + s], now + W + K + s, out=outs[W + K + s]),
                                  0, C_, world)
        lp = total_pkts + int(c2[268])
        long_h = {"steps": K + C_, "after_warmup": W, "mpps": round(lp / (elapsed + el2) / 1e6, 3),
                  "ms_per_step": round((elapsed + el2) / (K + C_) * 1e3, 4),
                  "continuation": {"steps": C_, "mpps": round(int(c2[268]) / el2 / 1e6, 3),
                                   "kernels_ms_per_step": kms(kern2, C_)}}
        log(f"long horizon: {long_h['mpps']} Mpps over {K + C_} steps (continuation {long_h['continuation']['mpps']})")
    local_pkts = sum(batches[s].n for s in range(W, W + K))
    if not os.environ.get("GPUFLOW_DIAG_LIB"):
        assert int(lc[268]) == local_pkts, (int(lc[268]), local_pkts)
    # roofline of the dominant kernel (k_ing_groups), this rank
    ki = kern.get("k_ing_groups", (0, 0.0))
    avg_ms = ki[1] / max(ki[0], 1)
    ranks = None
    if world > 1:
        # which rank set the max-over-ranks time, and what the counter all-reduce cost
        ranks = rank_diag(B, world, {"ms_per_step": B.local_elapsed / K * 1e3, "k_ing_groups_avg_ms": avg_ms,
                                     "counter_allreduce_ms": B.allreduce_ms, "packets": int(lc[268])})
    ab_per_launch = float(lc[270]) / max(K, 1)
    achieved = ab_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    cpu = par = None
    if not args.no_cpu:
        # every rank checks its own flow groups; the CPU baseline is rank 0's at N=1 only
        cpu, par = oracle_config2(args, B, sc, st, dp, batches, ps, outs, W, K, world, local_world, L, ct_names)
        if world > 1:
            cpu = None
    par = reduce_parity(B, par, rank, world)
    ct_end = sum(int(B.entries(dp, name)) for name in ct_names)
    B.close(dp)
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
                        "stream, 4M new flows/step (16M active), 256 endpoints, 4352 identities"
                        + (f", per-endpoint CT maps (ConntrackLocal, {len(ct_names)} maps)" if args.ct_local else ""),
            "packets_per_step_per_gpu": int(batches[W].n),
            "address_pairs_per_gpu": int(args.pairs),
            "address_pairs": int(args.pairs) * world,
            "ct_max_entries": int(ct_max),
            "ct_entries_at_end": ct_end,
            "parallelism": f"dp{world} (flow-group sharded, tables replicated, CT partitioned)",
        },
        "long_horizon": long_h and dict(long_h, ratio_to_headline=round(long_h["mpps"] / (total_pkts / elapsed / 1e6), 4)),
        "roofline": {
            "bound": "hbm",
            "kernel": "k_ing_groups (CT+policy stage: handle_policy over every packet of the step)",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "frac_source": "HIP events on the launch stream (this run)",
            "traffic": None,
            "algorithmic_bytes_per_launch": ab_per_launch,
            "avg_launch_ms": round(avg_ms, 4),
        },
        "kernels_ms_per_step": kms(kern, K),
        **({"ranks": ranks} if ranks else {}),
        "verdicts": verdicts(c),
        "cpu_baseline": cpu,
        "parity": par,
        **({"diag_writes_per_packet": {k: round(v / max(total_pkts, 1), 4) for k, v in wr.items()}} if wr else {}),
    }


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


def ct_local_split(sc, P, ct_max):
    """--ct-local: every endpoint binds a CT map of its own (the ConntrackLocal option,
    pkg/endpoint/bpf.go:268-276: cilium_ct4_<id>, max_entries ct_max / endpoints), holding
    the pre-inserted entries of its address (the tuple's daddr); the global map goes."""
    from cilium_amd import synth
    g = sc.maps.pop("cilium_ct4_global")
    ep_ip, lxc_id = np.asarray(P["ep_ip"], np.uint32), np.asarray(P["lxc_id"])
    order = np.argsort(ep_ip)
    d = g.keys[:, 0:4].copy().view(">u4").ravel().astype(np.uint32)
    pos = np.clip(np.searchsorted(ep_ip[order], d), 0, len(ep_ip) - 1)
    own = np.where(ep_ip[order][pos] == d, order[pos], -1)
    names = []
    per = max(1, ct_max // len(sc.lxc))
    for e in sc.lxc:
        j = int(np.nonzero(lxc_id == e["lxc_id"])[0][0])
        m = own == j
        name = f"cilium_ct4_{e['lxc_id']}"
        sc.add_map(synth.MapSpec(name, g.type, g.ksz, g.vsz, per, g.flags, g.keys[m], g.vals[m]))
        e["ct4"] = name
        names.append(name)
    return names


def oracle_config2(args, B, sc, st, dp, batches, ps, outs, W, K, world=1, local_world=1, L=None,
                   ct_names=("cilium_ct4_global",)):
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
    L = L or W + K
    T = cpu_threads(local_world)
    div = parity_div(args, world, T, sum(b.n for b in batches[:L]))
    t0 = time.time()
    ref = OracleDP(sc, shards=T)
    if div > 1:
        lru_replay(B, dp, ref)          # a sample cannot derive the whole table's cutoffs
    sa, da = st.p_saddr.cpu().numpy(), st.p_daddr.cpu().numpy()
    samp = torch.from_numpy(PY.pair_sampled(sa, da, div)).to(st.device)
    one = torch.from_numpy(PY.pair_sampled(sa, da, div * 8)).to(st.device)
    par = Parity(f"1/{div} of the address pairs (whole flow groups), every step incl. warm-up")
    done = single_n = 0
    tt = single_t = 0.0

    def host_step(s):                                   # frames + GPU records of step s, on the host
        idx = None if div == 1 else torch.nonzero(samp[ps[s]]).squeeze(1)
        pk = cols_packets(batches[s].cdict, idx)
        go = (outs[s] if idx is None else outs[s][idx]).cpu().numpy().view(ING_OUT).ravel()
        m1 = (one[ps[s]] if idx is None else one[ps[s]][idx]).cpu().numpy() if s == W else None
        return pk, go, m1
    import concurrent.futures as cf
    prep = cf.ThreadPoolExecutor(1)                     # step s+1 is prepared while the oracle runs step s
    nxt = prep.submit(host_step, 0)
    for s in range(L):
        pk, gout, m1 = nxt.result()
        if s + 1 < L:
            nxt = prep.submit(host_step, s + 1)
        if s == W:
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
            if W <= s < W + K:
                tt += time.perf_counter() - a
                done += pk.n
        par.records(gout, r, f"step {s}")
        if (s + 1) % 8 == 0:
            log(f"parity: {s + 1} of {L} steps, {par.packets} packets compared, {par.bad} mismatches "
                f"({time.time() - t0:.1f}s)")
    prep.shutdown()
    for name in ct_names:
        compare_ct(B, par, dp, ref, name, 14, div)
    ctl = par.ct if len(par.ct) <= 4 else {f"{len(par.ct)} maps": {k: sum(v[k] for v in par.ct.values())
                                                                  for k in ("entries_compared", "mismatches")}}
    log(f"cpu baseline + parity: {par.packets} packets compared, {par.bad} mismatches; CT {ctl}; "
        f"{done} packets in {tt:.2f}s on {T} threads ({time.time() - t0:.1f}s)")
    cpu = cpu_base(done / tt / 1e6 if tt else 0.0, T,
                   f"{done} packets of the same config-2 stream (flows of 1/{div} of the address pairs, the "
                   f"{K} timed steps after the same {W} warm-up steps), oracle restatement, RSS-style flow-group "
                   f"partition over {T} threads; single core: {single_n} packets of step {W}",
                   single_n / single_t / 1e6 if single_t else None)
    res = par.result(L)
    if len(res.get("tables", {})) > 4:                  # per-endpoint maps: one summary
        t = res["tables"]
        res["tables"] = {f"{len(t)} per-endpoint maps": {k: sum(v[k] for v in t.values())
                                                         for k in ("entries_compared", "mismatches", "gpu_entries_total")}}
    if div == 1:
        ev = {}
        for name in ct_names:
            dev_log = [tuple(int(x) for x in e) for e in B.evict_log(dp, name)]
            ora_log = [tuple(int(x) for x in e) for e in ref.lru_log.get(name, [])]
            ev[name] = {"evict_log_equal": dev_log == ora_log, "sweeps_device": len(dev_log),
                        "sweeps_oracle": len(ora_log), "entries_evicted": int(sum(e[5] for e in dev_log)),
                        "oracle": "own cutoffs from its whole table (never saw the device log)"}
        if len(ev) > 4:                                 # per-endpoint maps: one summary
            ev = {f"{len(ev)} per-endpoint maps": {
                "evict_log_equal": all(v["evict_log_equal"] for v in ev.values()),
                "sweeps_device": sum(v["sweeps_device"] for v in ev.values()),
                "sweeps_oracle": sum(v["sweeps_oracle"] for v in ev.values()),
                "entries_evicted": sum(v["entries_evicted"] for v in ev.values()),
                "oracle": "own cutoffs from each whole table (never saw the device logs)"}}
        res["evictions"] = ev
    return cpu, res


# Per-thread rate the parity budget assumes for the oracle (the config-2 CPU
# baseline ran 7.6 Mpps on 16 threads of the GPU box, 0.48 per thread: a margin
# below that) and the wall time one rank's parity leg may take at N>1.
ORACLE_MPPS_PER_THREAD = 0.4
PARITY_LEG_S = 60.0


def parity_div(args, world, threads=None, packets=None):
    """The flow-group sample of the parity legs: every pair at N=1 (the whole
    stream).  At N>1 the N oracles share one host: each rank checks 1/div of its
    own pairs, div >= 2 and large enough that `packets` (the rank's packets over
    the leg's steps) / div run within PARITY_LEG_S on its `threads` host threads
    (its share of the host's cores, cpu_threads(local_world))."""
    if args.parity_div:
        return args.parity_div
    if world == 1:
        return 1
    if not threads or not packets:
        return 2
    need = packets / (threads * ORACLE_MPPS_PER_THREAD * 1e6 * PARITY_LEG_S)
    return max(2, int(np.ceil(need)))


# ----------------------------------------------------------------------------- config 1 / 3 (stateless)
def bench_config1(args, B):
    import torch
    import ctypes as C
    from cilium_amd import synth
    from cilium_amd._lib import lib
    from cilium_amd.datapath import DeviceBatch
    sc = synth.config1()
    pk = sc.batches[0]
    dp = B.datapath(sc)
    b = DeviceBatch(pk)
    out = torch.empty(b.n, dtype=torch.uint8, device=B.dev)

    def step(s):
        c = b.cols()
        lib.gf_xdp_classify(dp.xdp_prog, C.byref(c), out.data_ptr(), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    W, K = 5, 50
    el, c, _, kern = timed(B, step, W, K)
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
    B.close(dp)
    return {"workload": "config1: bpf_xdp CIDR prefilter (10k LPM prefixes + 2k /32, 1025 endpoints), 1M packets/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_xdp"], float(c[270]) / K, "k_xdp", K), "kernels_ms_per_step": kms(kern, K),
            "verdicts": {"pass": int(c[258]), "drop": int(c[257])},
            "cpu_baseline": cpu, "parity": par}


def bench_config3(args, B):
    import torch
    import ctypes as C
    from cilium_amd import synth
    from cilium_amd._lib import lib
    from cilium_amd.datapath import DeviceBatch, LB_OUT
    sc = synth.config3(n_packets=16_000_000)
    pk = sc.batches[0]
    dp = B.datapath(sc)
    b = DeviceBatch(pk, with_v6=False)
    out = torch.empty((b.n, 12), dtype=torch.uint8, device=B.dev)

    def step(s):
        c = b.cols()
        lib.gf_lb_classify(dp.lb_prog, C.byref(c), out.data_ptr(), None,
                           C.c_void_p(torch.cuda.current_stream().cuda_stream))
    W, K = 3, 10
    el, c, _, kern = timed(B, step, W, K)
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
    B.close(dp)
    return {"workload": "config3: bpf_lb lb4_lookup_service + slave select, 100k services / ~1M backends, "
                        "16M packets/step (Zipf 1.1)",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, ["k_lb"], float(c[270]) / K, "k_lb", K), "kernels_ms_per_step": kms(kern, K),
            "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


# ----------------------------------------------------------------------------- config 4 (full pipeline)
class FrameBatch:
    def __init__(self, frames, lens, tc_index, dev, lxc_id=None, flow_hash=None):
        self.frames, self.len, self.tc_index, self.lxc_id, self.flow_hash = frames, lens, tc_index, lxc_id, flow_hash
        self.n, self.device = frames.shape[0], dev


def _spread(fb, samp, world):
    """The NIC side of the exchange-ingest leg (untimed): contiguous slice j of this
    rank's owned batch arrives on rank j, so every rank holds a mix of all ranks'
    flow groups, in arrival order, and must re-partition before classifying.  The
    sample bit travels with each frame (parity bookkeeping, not classifier input)."""
    import torch
    import torch.distributed as dist
    n = fb.n
    cuts = [n * j // world for j in range(world + 1)]
    send = [cuts[j + 1] - cuts[j] for j in range(world)]
    cnt = torch.tensor(send, dtype=torch.int64, device=fb.frames.device)
    recv_cnt = torch.empty_like(cnt)
    dist.all_to_all_single(recv_cnt, cnt)
    recv = recv_cnt.cpu().tolist()
    out = []
    for t in (fb.frames, fb.len, fb.tc_index, samp):
        r = torch.empty((sum(recv),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(r, t.contiguous(), recv, send)
        out.append(r)
    return FrameBatch(out[0], out[1], out[2], fb.device), out[3]


def bench_config4(args, B, rank=0, world=1, ingest="owned", local_world=1):
    """BASELINE config 4 over raw frames.  ingest "owned": each rank's frames are
    the packets of its own flow groups (the RSS of a NIC programmed with the owner
    hash); "exchange" (N>1): frames arrive anywhere and each step first runs
    gf_pipeline_partition + one all-to-all (cilium_amd.shard, RCCL over xGMI) —
    inside the timed region."""
    import torch
    from cilium_amd import synth, stream
    from oracle import parity as PY
    W = 4
    K = max(4, args.c4_steps - W) if args.c4_steps else max(4, args.steps // 2)
    ct_max = min(args.ct_max, B.ct_max_cap or args.ct_max)
    kw = dict(B.tables_kw, n_svc=1000, n_lpm=500, n_fix=100) if B.rehearsal else {}
    sc, P, vip = synth.config4_tables(n_pairs=args.pairs * world, ct_max=ct_max, **kw)
    st = stream.Stream(P, rank=rank, world=world, flows_per_step=args.flows_per_step, device=B.dev, vip_ip=vip)
    S0 = 3
    rk, rv = st.reply_ct_entries(S0 + W + K)
    sc.maps["cilium_ct4_global"].keys, sc.maps["cilium_ct4_global"].vals = rk, rv
    dp = B.datapath(sc)
    exch = ingest == "exchange" and world > 1
    # N=1: the whole stream (every packet, the whole CT, the oracle's own eviction
    # cutoffs); N>1: the pipeline oracle is ~2x the per-packet cost of ingress, half
    # the per-rank sample
    div = parity_div(args, world, cpu_threads(local_world), 2 * (W + K) * args.flows_per_step * 4)
    if world > 1 and not args.parity_div:
        div *= 2
    # steps whose rewritten frames are fingerprinted on the device (snap_out) and
    # compared with the oracle's: the warm-up steps (untimed) by default, every
    # step with --c4-frames all (then the timed steps also write the snaps)
    fp_steps = {"none": 0, "warmup": W, "all": W + K}[args.c4_frames] if not args.no_cpu else 0
    fps = [None] * (W + K)
    sa, da = st.p_saddr.cpu().numpy(), st.p_daddr.cpu().numpy()
    pm = torch.from_numpy(PY.pair_sampled(sa, da, div).astype(np.uint8) |
                          (PY.pair_sampled(sa, da, div * 8).astype(np.uint8) << 1)).to(B.dev)
    fbs, ps, samps = [], [], []
    for s in range(W + K):
        cols, p, n = st.step(S0 + s)
        f, lens = stream.device_frames(cols)
        fb = FrameBatch(f, lens, cols["tc_index"], B.dev)
        sm = pm[p]
        if exch:
            fb, sm = _spread(fb, sm, world)
        fbs.append(fb)
        ps.append(p)
        samps.append(sm)
    B.sync()
    got = [None] * (W + K)            # exchange: the batch each step classified (its records' order)

    if exch:
        from cilium_amd import shard

        def step(s):
            fb = fbs[s]
            owner, order, counts = B.partition(dp, fb, rank, world)
            fr, ln, tc, sm = shard.exchange(order, counts, [fb.frames, fb.len, fb.tc_index, samps[s]])
            mine = FrameBatch(fr, ln, tc, B.dev)
            out = torch.empty((mine.n, 24), dtype=torch.uint8, device=B.dev)
            dp.pipeline(mine, sc.now + s, out=out, snap_out=False)
            got[s] = (mine, sm, out)
    else:
        outs = [torch.empty((b.n, 24), dtype=torch.uint8, device=B.dev) for b in fbs]

        def step(s):
            _, _, snap = dp.pipeline(fbs[s], sc.now + s, out=outs[s], snap_out=s < fp_steps)
            if snap is not None:
                fps[s] = PY.frame_fingerprints_torch(snap)
            got[s] = (fbs[s], samps[s], outs[s])
    el, c, lc, kern = timed(B, step, W, K, world)
    names = [k for k in kern]
    ranks = None
    if world > 1:
        ki = kern.get("k_ing_groups", (0, 0.0))
        ranks = rank_diag(B, world, {"ms_per_step": B.local_elapsed / K * 1e3,
                                     "k_ing_groups_avg_ms": ki[1] / max(ki[0], 1),
                                     "counter_allreduce_ms": B.allreduce_ms, "packets": int(lc[268])})
    cpu = par = None
    if not args.no_cpu:
        cpu, par = oracle_config4(args, B, sc, dp, got, W, K, div, local_world=local_world, replay=div > 1, fps=fps)
        if world > 1:
            cpu = None
    par = reduce_parity(B, par, rank, world)
    B.close(dp)
    r = {"workload": "config4: bpf_xdp -> bpf_lb -> bpf_netdev delivery -> handle_policy over raw 64-B frames "
                     "(config-2 stream, 30% of pairs via service VIPs; 10k-prefix prefilter; config 3's 100k "
                     "services / ~1M backends in the lbmap), 16.8M packets/step per GPU",
         "ingest": ("frames arrive on any rank; gf_pipeline_partition + RCCL all-to-all re-partition them by "
                    "post-LB flow group inside the timed step") if exch else
                   "frames arrive on the rank that owns their flow group (RSS by the owner hash)",
         "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
         "packets_per_step": int(c[268]) // K, "warmup": W, "n_gpus": world,
         **({"note": "--c4-frames all: every timed step also writes and fingerprints its rewritten frames "
                     "(a parity run, not the configuration's throughput)"} if fp_steps > W else {}),
         "roofline": roofline(kern, [k for k in names if k != "k_partition"], float(lc[270]) / K,
                              "all pipeline kernels (frames -> verdicts), this rank", K),
         "kernels_ms_per_step": kms(kern, K), **({"ranks": ranks} if ranks else {}),
         "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}
    if world == 1 and not B.rehearsal and not args.no_h2d:
        r["h2d"] = config4_h2d(args, B, sc, fbs, [g[2] for g in got], W, K)
    return r


def oracle_config4(args, B, sc, dp, got, W, K, div, ct_names=("cilium_ct4_global",), local_world=1, replay=True,
                   fps=None):
    """The oracle pipeline over the flow-group sample of every step (the flow group
    is the post-LB address pair, i.e. the stream's pair), records and the sampled
    pairs' CT entries compared; timed steps give the CPU baseline.  got[s] = (the
    frames step s classified, their sample bits, their records); sample bit 0: the packet's
    post-LB pair is in the 1/div sample, bit 1: in the 1/(8 div) single-core subsample.
    replay=False (div must be 1: the oracle holds the whole table): the oracle's LRU
    stand-in derives its own eviction cutoffs from its own table, and its eviction
    log must equal the device's (gf_ct_evict_log) entry for entry.  fps[s] (device
    int64 tensor or None): the fingerprints of step s's rewritten frames
    (oracle.parity.frame_fingerprints), compared with those of the oracle's frames."""
    import torch
    from cilium_amd.datapath import PIPE_OUT
    from cilium_amd.synth import Packets
    from oracle.scenario import OracleDP
    from oracle import parity as PY
    T = cpu_threads(local_world)
    ref = OracleDP(sc, shards=T)
    fr_n = fr_bad = 0
    fr_first = None
    if replay:
        lru_replay(B, dp, ref)
    else:
        assert div == 1, "independent eviction needs the whole table"
    par = Parity(f"1/{div} of the address pairs (whole flow groups), every step incl. warm-up")
    done = single_n = 0
    tt = single_t = 0.0
    for s in range(W + K):
        b, sm, out = got[s]
        sbits = sm.cpu().numpy()
        idx = np.nonzero(sbits & 1)[0]
        it = torch.from_numpy(idx).to(b.frames.device)
        pk = Packets(b.frames[it].cpu().numpy(), b.len[it].cpu().numpy().view(np.uint32),
                     tc_index=None if b.tc_index is None else b.tc_index[it].cpu().numpy())
        gout = out[it].cpu().numpy().view(PIPE_OUT).ravel()
        if s == W:
            # 1/8 of the sampled groups (sample bit 1) on one core first (exact: groups are independent)
            m1 = (sbits[idx] & 2) != 0
            a = time.perf_counter()
            o1 = ref.pipeline(_sub(pk, np.nonzero(m1)[0]), sc.now + s, threads=1, lru=False)
            single_t, single_n = time.perf_counter() - a, int(m1.sum())
            a = time.perf_counter()
            o2 = ref.pipeline(_sub(pk, np.nonzero(~m1)[0]), sc.now + s, threads=T)
            tt += time.perf_counter() - a
            done += pk.n - single_n
            r = np.empty(pk.n, o1[0].dtype)
            r[m1], r[~m1] = o1[0], o2[0]
            rs = np.empty((pk.n,) + o1[2].shape[1:], o1[2].dtype)
            rs[m1], rs[~m1] = o1[2], o2[2]
        else:
            a = time.perf_counter()
            o = ref.pipeline(pk, sc.now + s, threads=T)
            r, rs = o[0], o[2]
            if s >= W:
                tt += time.perf_counter() - a
                done += pk.n
        par.records(gout, r, f"step {s}")
        if fps is not None and fps[s] is not None:
            gf = fps[s][it].cpu().numpy().view(np.uint64)
            bad = np.nonzero(gf != PY.frame_fingerprints(rs))[0]
            fr_n += len(gf)
            fr_bad += len(bad)
            if len(bad) and fr_first is None:
                fr_first = f"step {s} sampled row {int(bad[0])}"
        if (s + 1) % 8 == 0:
            log(f"config-4 parity: {s + 1} of {W + K} steps, {par.packets} packets, {par.bad} mismatches, "
                f"{fr_n} frames, {fr_bad} frame mismatches")
    for name in ct_names:
        compare_ct(B, par, dp, ref, name, 14 if "4" in name else 40, div)
    cpu = cpu_base(done / tt / 1e6 if tt else 0.0, T,
                   f"{done} packets (flows of 1/{div} of the address pairs, the {K} timed steps after the same "
                   f"warm-up), {T} threads; single core: {single_n} packets of step {W}",
                   single_n / single_t / 1e6 if single_t else None)
    res = par.result(W + K)
    if fr_n:
        res["frames_compared"], res["frame_mismatches"] = int(fr_n), int(fr_bad)
        res["frames"] = ("64-bit fingerprints of the rewritten frames (snap_out; oracle.parity.frame_fingerprints), "
                         "device vs oracle, on the steps that wrote them")
        if fr_first:
            res["first_frame_mismatch"] = fr_first
    if not replay:
        for name in ct_names:
            dev_log = [tuple(int(x) for x in e) for e in B.evict_log(dp, name)]
            ora_log = [tuple(int(x) for x in e) for e in ref.lru_log.get(name, [])]
            res.setdefault("evictions", {})[name] = {
                "evict_log_equal": dev_log == ora_log, "sweeps_device": len(dev_log), "sweeps_oracle": len(ora_log),
                "entries_evicted": int(sum(e[5] for e in dev_log)),
                "oracle": "own cutoffs from its whole table (never saw the device log)"}
    return cpu, res



def config4_h2d(args, B, sc, fbs, outs, W, K):
    """Config 4 with the host->device copy of the frames in the timed region:
    each step's 64-B frames start in pinned host memory and are copied over PCIe
    on a copy stream (double-buffered: step s+1's copy runs under step s's
    kernels).  A fresh datapath over the same steps; its records must equal the
    device-resident run's bit for bit (same kernels, same state sequence)."""
    import torch
    t0 = time.time()
    W, K = 2, min(K, 4)                    # the first W + K steps of the device-resident run (pinned host copies)
    dp = B.datapath(sc)
    n = fbs[0].n
    host = [[t.cpu().pin_memory() for t in (fb.frames, fb.len, fb.tc_index)] for fb in fbs[:W + K]]
    dbuf = [[torch.empty_like(t) for t in (fbs[0].frames, fbs[0].len, fbs[0].tc_index)] for _ in range(2)]
    copy = torch.cuda.Stream()
    comp = torch.cuda.current_stream()
    ready = [torch.cuda.Event() for _ in range(2)]
    free = [torch.cuda.Event() for _ in range(2)]
    outs2 = [torch.empty((n, 24), dtype=torch.uint8, device=B.dev) for _ in range(W + K)]

    def issue_copy(s):
        j = s % 2
        with torch.cuda.stream(copy):
            copy.wait_event(free[j])
            for d, h in zip(dbuf[j], host[s]):
                d.copy_(h, non_blocking=True)
            ready[j].record(copy)

    def run(a, b):
        issue_copy(a)
        for s in range(a, b):
            if s + 1 < b:
                issue_copy(s + 1)
            j = s % 2
            comp.wait_event(ready[j])
            f, ln, tc = dbuf[j]
            dp.pipeline(FrameBatch(f, ln, tc, B.dev), sc.now + s, out=outs2[s], snap_out=False)
            free[j].record(comp)
    for j in range(2):
        free[j].record(comp)
    el, c, _, kern = timed(B, run, W, K, ranged=True)
    B.sync()
    same = all(torch.equal(outs[s], outs2[s]) for s in range(W + K))
    B.close(dp)
    byts = sum(t.numel() * t.element_size() for t in host[0])
    log(f"config 4 + H2D: {int(c[268]) / el / 1e6:.1f} Mpps, records equal the device-resident run: {same} "
        f"({time.time() - t0:.1f}s)")
    return {"mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "pcie_bytes_per_step": byts, "pcie_gbs": round(byts / (el / K) / 1e9, 2),
            "records_equal_device_resident": bool(same),
            "note": "frames + len + tc_index copied host->device every step (69 B/packet, pinned, double-buffered "
                    "on a copy stream); "
                    "reported beside the device-resident figure, never as the line's value"}


# ----------------------------------------------------------------------------- config 5 (IPv6 pipeline)
def bench_config5(args, B):
    """BASELINE config 5 through the path an IPv6 packet takes on a node: bpf_xdp's
    check_v6 (v6_dyn LPM, 10k /32-/127 prefixes; v6_fix hash, 100k /128s; endpoint
    check) -> bpf_netdev handle_ipv6 (identity from the flow label of cluster
    sources, hop limit, MACs) -> handle_policy / ipv6_policy with ct_lookup6 on a
    10,485,760-entry LRU CT pre-filled to 8M entries."""
    import torch
    from cilium_amd import synth, stream
    from oracle import parity as PY
    W, K = 3, 4
    t0 = time.time()
    sc, P, meta = synth.config5_tables(n_pairs=args.pairs, prefill=args.ct6_prefill, ct6_max=args.ct6_max)
    st = stream.Stream6Frames(P, meta, flows_per_step=args.c5_flows, device=B.dev)
    S0 = 3
    rk, rv = st.reply_ct6_entries(S0 + W + K)
    ct6 = sc.maps["cilium_ct6_global"]
    ct6.keys, ct6.vals = synth.ct6_prefill(meta, rk, rv, sc.now)
    dp = B.datapath(sc)
    log(f"config5: tables + {sc.maps['cilium_ct6_global'].n()} pre-filled CT6 entries ({time.time() - t0:.1f}s)")
    # the whole stream: the oracle holds the whole CT6, so its LRU stand-in evicts on
    # its own cutoffs and its eviction log is compared with the device's
    div = 1
    a6, b6 = st.pair_addrs6()
    pm = torch.from_numpy(PY.pair_sampled6(a6, b6, div).astype(np.uint8) |
                          (PY.pair_sampled6(a6, b6, div * 8).astype(np.uint8) << 1)).to(B.dev)
    fbs, got = [], []
    for s in range(W + K):
        f, lens, p = st.step(S0 + s)
        fbs.append(FrameBatch(f, lens, None, B.dev))
        got.append((fbs[-1], pm[p], torch.empty((f.shape[0], 24), dtype=torch.uint8, device=B.dev)))
    B.sync()
    el, c, _, kern = timed(B, lambda s: dp.pipeline(fbs[s], sc.now + s, out=got[s][2], snap_out=False), W, K)
    names = [k for k in kern]
    cpu = par = None
    if not args.no_cpu:
        cpu, par = oracle_config4(args, B, sc, dp, got, W, K, div, ct_names=("cilium_ct6_global",), replay=False)
    ct6_end, evictions = int(B.entries(dp, "cilium_ct6_global")), len(B.evict_log(dp, "cilium_ct6_global"))
    B.close(dp)
    return {"workload": "config5: IPv6 bpf_xdp check_v6 (10k v6_dyn /32-/127 + 100k v6_fix /128) -> bpf_netdev "
                        f"handle_ipv6 -> handle_policy ipv6_policy (ct_lookup6), CT6 max {args.ct6_max:,} (LRU) pre-filled "
                        f"to {args.ct6_prefill}, {args.c5_flows} new flows/step",
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "ct6_entries_at_end": ct6_end,
            "ct6_evictions": evictions,
            "roofline": roofline(kern, names, float(c[270]) / K, "all pipeline kernels (frames -> verdicts)", K),
            "kernels_ms_per_step": kms(kern, K), "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


# ----------------------------------------------------------------------------- endpoint egress
def bench_egress(args, B):
    """The from-container program (handle_ipv4_from_lxc) over frames sent by 256
    local endpoints (synth.TENANT per tenant), local deliveries continuing into handle_policy:
    4M flows, one 64-B frame each per step; each step a quarter of the flows
    starts anew (new source port), the rest are established."""
    import torch
    from cilium_amd import synth
    W, K = 3, max(4, args.steps // 2)
    n = args.egress_flows
    t0 = time.time()
    sc, meta = synth.egress_tables(ct_max=args.ct_max)
    ct_names = ["ct4"]
    if args.ct_local:                                   # every endpoint on CT maps of its own (ConntrackLocal)
        made = synth.conntrack_local(sc, max_entries=max(1, args.ct_max // len(sc.lxc)))
        sc.maps.pop("ct4", None)
        sc.maps.pop("ct6", None)
        ct_names = [m for m in made if m.startswith("ct4_")]
    f, lens, lid, fh = synth.egress_flows(meta, n)
    dp = B.datapath(sc)
    log(f"egress: tables and {n} flows ({time.time() - t0:.1f}s)")
    base = torch.from_numpy(f).to(B.dev)
    q = n // 4
    frames = []
    for s in range(W + K):
        fs = base.clone()
        a = (s % 4) * q                    # a new source port for each flow of this quarter
        sp = base[a:a + q, 34].to(torch.int64) * 256 + base[a:a + q, 35].to(torch.int64)
        sp = 1024 + (sp - 1024 + 7919 * (s + 1)) % 60000
        fs[a:a + q, 34], fs[a:a + q, 35] = (sp >> 8).to(torch.uint8), (sp & 0xff).to(torch.uint8)
        frames.append(fs)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(B.dev)
    len_t, lid_t, fh_t = t(lens, np.int32), t(lid, np.int16), t(fh, np.int32)
    fbs = [FrameBatch(frames[i], len_t, None, B.dev, lid_t, fh_t) for i in range(W + K)]
    outs = [torch.empty((n, 24), dtype=torch.uint8, device=B.dev) for _ in range(W + K)]
    el, c, _, kern = timed(B, lambda s: dp.egress(fbs[s], sc.now + s, out=outs[s], snap_out=False), W, K)
    log(f"egress: timed {K} steps ({time.time() - t0:.1f}s)")
    cpu = par = None
    if not args.no_cpu:
        cpu, par = oracle_egress(args, B, sc, meta, dp, frames, lens, lid, fh, outs, W, K, ct_names)
    B.close(dp)
    return {"workload": "egress: bpf_lxc from-container handle_ipv4_from_lxc (+ handle_policy of local deliveries), "
                        f"256 endpoints, {n} flows/step (35% world, 20% tunnel, 25% local, 20% service "
                        "VIPs), 1/4 new per step"
                        + (f", per-endpoint CT maps (ConntrackLocal, {len(ct_names)} CT4 maps)" if args.ct_local else ""),
            "mpps": round(int(c[268]) / el / 1e6, 1), "ms_per_step": round(el / K * 1e3, 4), "steps": K,
            "packets_per_step": int(c[268]) // K, "warmup": W,
            "roofline": roofline(kern, list(kern), float(c[270]) / K, "all egress kernels (frames -> verdicts)", K),
            "kernels_ms_per_step": kms(kern, K), "verdicts": verdicts(c), "cpu_baseline": cpu, "parity": par}


def oracle_egress(args, B, sc, meta, dp, frames, lens, lid, fh, outs, W, K, ct_names=("ct4",)):
    """Parity and the CPU baseline from one pass: T oracle instances side by side,
    one per closed share of the flow groups (a tenant's local and service flows
    stay together; flows to world and tunnel peers, whose CT keys are their own
    address pair, spread by pair hash), each running its share of every step
    packet by packet.  Every packet's record is compared with the GPU's, and the
    union of the instances' CT tables with the GPU's whole CT.  The shares are
    exact for this workload because no CT key, proxy entry or LRU eviction is
    shared between them: the egress CT stays far below max_entries (the GPU's
    eviction log is checked to be empty; otherwise one sequential oracle runs
    every packet instead, as before).  The timed steps of the same pass give the
    CPU baseline."""
    import threading
    import torch
    from cilium_amd.datapath import EG_OUT
    from cilium_amd.synth import Packets, TENANT
    from oracle.scenario import OracleDP
    from oracle import parity as PY
    ep_idx = lid.astype(np.int64) - int(meta["lxc_id"][0])
    ten = ep_idx // TENANT
    T = cpu_threads()
    evicted = any(len(B.evict_log(dp, name)) for name in ct_names)
    if evicted:
        T = 1                                           # LRU evictions depend on the whole table: one instance
    f0 = frames[0].cpu().numpy()
    dst = f0[:, 30:34].copy().view(">u4").ravel()
    src_raw, dst_raw = f0[:, 26:30].copy().view("<u4").ravel(), f0[:, 30:34].copy().view("<u4").ravel()
    inside = ((dst >> 16) == 0x0a01) | ((dst >> 16) == 0x0a60)          # endpoints 10.1/16, service VIPs 10.96/16
    hsh = (PY._fmix64((np.maximum(src_raw, dst_raw).astype(np.uint64) << np.uint64(32)) |
                      np.minimum(src_raw, dst_raw).astype(np.uint64)) % np.uint64(T)).astype(np.int64)
    owner = np.where(inside, ten % T, hsh)
    shares = [np.nonzero(owner == t)[0] for t in range(T)]
    insts = [OracleDP(sc) for _ in range(T)]
    for ref in insts:
        lru_replay(B, dp, ref)
    par = Parity(f"every packet of every step, {T} oracle instances over closed flow-group shares"
                 if T > 1 else "every packet of every step, one sequential oracle")
    tt, done = 0.0, 0
    for s in range(W + K):
        host = frames[s].cpu().numpy()
        recs = [None] * T

        def run(t):
            sh = shares[t]
            recs[t], _ = insts[t].egress(Packets(host[sh], lens[sh], None, None, lid[sh], None, fh[sh]), sc.now + s)
        th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        a = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        if s >= W:
            tt += time.perf_counter() - a
            done += len(lid)
        r = np.empty(len(lid), recs[0].dtype)
        for t in range(T):
            r[shares[t]] = recs[t]
        par.records(outs[s].cpu().numpy().view(EG_OUT).ravel(), r, f"step {s}")
    for name in ct_names:                               # (each map: the union of the instances' copies)
        gk, gv, gtot = B.table_sampled(dp, name, 14, 1, lambda k, div: np.ones(len(k), bool))
        dumps = [ref.m[name].dump_arrays() for ref in insts]
        rk = np.concatenate([d[0] for d in dumps]) if dumps else np.zeros((0, 14), np.uint8)
        rv = np.concatenate([d[1] for d in dumps]) if dumps else np.zeros((0, 48), np.uint8)
        par.table(name, gk, gv, rk, rv, gtot)
    one = OracleDP(sc)
    sh = shares[0][: max(1, len(shares[0]) // 4)]
    host0 = frames[0].cpu().numpy()
    a = time.perf_counter()
    one.egress(Packets(host0[sh], lens[sh], None, None, lid[sh], None, fh[sh]), sc.now)
    t1 = time.perf_counter() - a
    cpu = cpu_base(done / tt / 1e6 if tt else 0.0, T,
                   f"{done} packets (every flow of the {K} timed steps after {W} warm-up steps), {T} oracle instances "
                   f"over closed flow-group shares; single core: {len(sh)} frames of step 0",
                   len(sh) / t1 / 1e6 if t1 else None)
    res = par.result(W + K)
    if len(res.get("tables", {})) > 4:                  # per-endpoint maps: one summary
        t = res["tables"]
        res["tables"] = {f"{len(t)} per-endpoint maps": {k: sum(v[k] for v in t.values())
                                                         for k in ("entries_compared", "mismatches", "gpu_entries_total")}}
    return cpu, res


EXTRA = {"1": bench_config1, "3": bench_config3, "4": bench_config4, "5": bench_config5, "egress": bench_egress}


# Issue and memory-operation ceilings the roofline objects are also priced against
# (the byte roofline alone names the wrong bound for a kernel of random accesses,
# DESIGN.md §6), all measured on MI355X by tools/primbench.hip
# (profiles/r4_primbench.txt, request sizes in profiles/r4_primbench_pmc.txt):
#   issue:   VALU + SALU wave-instructions per second / (256 CUs x 4 SIMDs x 2.4 GHz)
#            ("valu_busy" = 2 x VALU / the same: a wave64 VALU holds its SIMD-32 2 clocks)
#   memory:  per operation kind, its rate over the kernel's launch time against the
#            best rate of that kind measured for random addresses over a 16-GB table:
#            128-B line reads (every random read fills a whole 128-B L2 line) 54 G/s
#            (nontemporal 16-B loads), partial (32-B) writes 21.7 G/s, full 64-B line
#            writes 60.5 G/s (four lanes one 16-B store each), u64 atomics 17.3 G/s.
#            frac = the largest of the four: the kind closest to its own ceiling.
ISSUE_PEAK = 256 * 4 * 2.4e9
MEM_CEIL = {"line_reads": 54.0e9, "partial_writes": 21.7e9, "full_writes_64B": 60.5e9, "atomics": 17.3e9}
PMC_ROUND = "r6"          # the round whose per-kernel PMC summaries price this run (built from the same sources)
PMC_KERNELS = {"2": ["k_ing_groups"], "1": ["k_xdp", "k_xdp_lds"], "3": ["k_lb"]}   # else: every kernel


def add_bounds(cfg, r):
    """roofline.traffic / .issue / .memory of configuration `cfg` from this round's
    per-kernel PMC summary (profiles/<PMC_ROUND>_pmc_kernels_c<cfg>.json,
    tools/pmc_kernels.py), scaled per packet to this run and divided by this run's
    live launch time.  Only a summary built from the library this run loaded
    (same gf_build_id) is used; otherwise the bound is marked stale."""
    rf = r.get("roofline")
    path = os.path.join(ROOT, "profiles", f"{PMC_ROUND}_pmc_kernels_c{cfg}.json")
    if not rf or not rf.get("avg_launch_ms"):
        return r
    if not os.path.exists(path):
        rf["bounds_source"] = f"missing: {os.path.relpath(path, ROOT)}"
        return r
    try:
        j = json.load(open(path))
        src = os.path.relpath(path, ROOT)
        try:
            from cilium_amd import _lib
            built = _lib.BUILD_ID
        except Exception:
            built = None
        if j.get("build_id") != built:
            rf["bounds_stale"] = {"source": src, "summary_build_id": j.get("build_id"), "library_build_id": built}
            return r
        names = PMC_KERNELS.get(cfg) or [k for k in j["kernels"] if k.startswith("k_") or k == "rocprim"]
        ks = [j["kernels"][k] for k in names if k in j["kernels"]]
        pk = r.get("packets_per_step") or r.get("config", {}).get("packets_per_step_per_gpu")
        scale = float(pk) / float(j["packets_per_step"])
        t = rf["avg_launch_ms"] * 1e-3
        cs = lambda n: sum(k["counters_per_step"].get(n, 0.0) for k in ks) * scale
        valu, salu = cs("SQ_INSTS_VALU"), cs("SQ_INSTS_SALU")
        if valu or salu:
            rf["issue"] = {"frac": round((valu + salu) / t / ISSUE_PEAK, 4),
                           "valu_busy": round(2 * valu / t / ISSUE_PEAK, 4),
                           "wave_insts_per_s": (valu + salu) / t, "peak": ISSUE_PEAK,
                           "wave_insts_per_64_packets": round((valu + salu) * 64 / float(pk), 1), "source": src}
        # the same algorithmic bytes over the profiled run's own kernel average
        # (rocprofv3 --stats of this build), beside the live HIP-event frac
        ns = [k.get("rocprof_avg_ns") for k in ks]
        ab = rf.get("algorithmic_bytes_per_launch")
        if ab and ns and all(ns):
            ms_p = sum(k["rocprof_avg_ns"] * k.get("dispatches_per_step", 1.0) for k in ks) * 1e-6
            # one frac per line: the profile's (the rocprofv3 --stats average this line
            # cites), so frac = algorithmic_bytes_per_launch / rocprof_avg_launch_ms
            # reproduces from profiles/; the live HIP-event figure stays beside it
            rf["frac_hip_events"], rf["achieved_hip_events"] = rf["frac"], rf["achieved"]
            rf["achieved"] = round(ab / (ms_p * 1e-3) / 1e9, 2)
            rf["frac"] = rf["frac_rocprof"] = round(ab / (ms_p * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            rf["frac_source"] = ("algorithmic_bytes_per_launch / rocprof_avg_launch_ms (rocprofv3 --kernel-trace "
                                 "--stats of this build: rocprof_source)")
            rf["rocprof_avg_launch_ms"] = round(ms_p, 4)
            rf["rocprof_source"] = j.get("kernel_stats_source", src)
        tb = sum(k.get("traffic_bytes_per_packet") or 0.0 for k in ks) * float(pk)
        if tb:
            rf["traffic"] = tb
            rf["traffic_kind"] = ("EA-request bytes (MALL hits included): L2->fabric requests priced by their size, "
                                  "not DRAM bytes")
            rf["traffic_source"] = src
            rf["traffic_model"] = ks[0].get("traffic_model") if ks else None
            hits = cs("TCC_HIT_sum")
            miss = cs("TCC_MISS_sum")
            if hits + miss:
                rf["l2_hit_rate"] = round(hits / (hits + miss), 4)
        per = {}
        for k in ks:
            for n_, v in (k.get("per_packet") or {}).items():
                per[n_] = per.get(n_, 0.0) + v
        if per:
            mem = {"source": src, "ceilings_source": "profiles/r4_primbench.txt", "per_packet": per}
            fr = {}
            for n_, ceil in MEM_CEIL.items():
                rate = per.get(n_, 0.0) * float(pk) / t
                fr[n_] = {"per_s": rate, "ceiling": ceil, "frac": round(rate / ceil, 4)}
            mem["kinds"] = fr
            bind = max(fr, key=lambda n_: fr[n_]["frac"])
            mem["frac"], mem["binding"] = fr[bind]["frac"], bind
            rf["memory"] = mem
    except Exception as e:                                   # reported, never silently dropped
        rf["bounds_error"] = f"{type(e).__name__}: {e}"
    return r


# ----------------------------------------------------------------------------- launcher (--gpus N)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus():
    """GPUs this process may use, counted without the HIP runtime (the launcher
    must not initialise the GPU before it starts the ranks): the device lists of
    HIP/ROCR/CUDA_VISIBLE_DEVICES when set, else the GPU nodes of the KFD
    topology (/sys/class/kfd/kfd/topology/nodes/*/gpu_id != 0)."""
    lists = [os.environ[v] for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
             if v in os.environ]
    if lists:
        return min(len([x for x in v.split(",") if x.strip() not in ("", "-1")]) for v in lists)
    n = 0
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            with open(p) as f:
                n += int(f.read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    return n


def spawn_ranks(n, argv):
    """`bench.py --gpus N` run directly (no torch.distributed launcher): start the N
    rank processes (each child pins LOCAL_RANK) before this process has imported
    torch or touched the HIP runtime, wait for all, return the worst exit status."""
    vis = visible_gpus()
    if n > vis and not os.environ.get("GPUFLOW_BENCH_SHARE_GPU"):
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
    ap.add_argument("--long-steps", type=int, default=64,
                    help="config 2 at N=1: steps in all (warm-up + timed + a timed continuation into LRU eviction)")
    ap.add_argument("--ct6-max", type=int, default=10_485_760, help="config 5: CT6 max_entries (LRU)")
    ap.add_argument("--c5-flows", type=int, default=1 << 20, help="config 5: new flows per step")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and the parity legs")
    ap.add_argument("--pipeline", action="store_true",
                    help="config 2: the steps through gf_policy_ingress_classify_batches (schedule overlap)")
    ap.add_argument("--no-extra", action="store_true", help="config 2 only (skip the other configurations)")
    ap.add_argument("--no-h2d", action="store_true", help="config 4: skip the leg with the host->device copy")
    ap.add_argument("--ct-local", action="store_true",
                    help="configs 2 and egress: every endpoint on CT maps of its own (the ConntrackLocal option)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--parity-div", type=int, default=0,
                    help="parity sample: 1 in N address pairs (default: every pair at N=1, 1 in 2 per rank at N>1)")
    ap.add_argument("--egress-flows", type=int, default=4 << 20)
    ap.add_argument("--c4-steps", type=int, default=0,
                    help="config 4: steps in all, warm-up included (default: 4 + max(4, --steps / 2))")
    ap.add_argument("--c4-frames", default="warmup", choices=["none", "warmup", "all"],
                    help="config 4: steps whose rewritten frames are fingerprinted and compared with the oracle's")
    args = ap.parse_args()

    rehearsal = bool(os.environ.get("GPUFLOW_BENCH_SELFTEST"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        log(f"WORLD_SIZE {world} != --gpus {args.gpus}: the launcher's world size is used")

    import torch.distributed as dist
    if rehearsal:
        B = Rehearsal()
        if world > 1:
            dist.init_process_group("gloo")
    else:
        B = Gpu(local)
        if world > 1:
            backend = os.environ.get("GPUFLOW_BENCH_BACKEND", "nccl")      # nccl = RCCL over xGMI
            dist.init_process_group(backend, **({"device_id": B.dev} if backend == "nccl" else {}))

    if args.config == "2":
        res = add_bounds("2", bench_config2(args, B, rank, world, local_world))
        extra = {} if args.no_extra else (
            {k: v for k, v in EXTRA.items()} if world == 1 and not rehearsal else
            {"4": lambda a, b: bench_config4(a, b, rank, world, "owned", local_world),
             "4x": lambda a, b: bench_config4(a, b, rank, world, "exchange", local_world)} if world > 1 else
            {"4": lambda a, b: bench_config4(a, b, rank, world, "owned", local_world)})
        if extra:
            res["configs"] = {}
        for k, fn in extra.items():
            t0 = time.time()
            try:
                res["configs"][k] = add_bounds(k, fn(args, B))
            except Exception as e:                       # reported, never silently dropped
                if world > 1:
                    raise                                # a rank cannot skip a collective the others run
                res["configs"][k] = {"error": f"{type(e).__name__}: {e}"}
            log(f"config {k}: {res['configs'][k].get('mpps')} Mpps ({time.time() - t0:.1f}s)")
            if not rehearsal:
                import torch
                torch.cuda.empty_cache()
    else:
        if world > 1 and args.config != "4":
            raise SystemExit("--config other than 2 and 4 runs on one GPU")
        if args.config == "4":
            r = bench_config4(args, B, rank, world, "owned", local_world)
        else:
            r = EXTRA[args.config](args, B)
        r = add_bounds(args.config, r)
        res = {"metric": METRIC, "value": r["mpps"], "unit": "Mpps", "n_gpus": world, "steps": r["steps"],
               "warmup": r["warmup"], "ms_per_step": r["ms_per_step"], "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "u32", "data": "synthetic",
               "config": {"workload": r["workload"], "packets_per_step": r["packets_per_step"]},
               "roofline": r["roofline"], "kernels_ms_per_step": r["kernels_ms_per_step"],
               "cpu_baseline": r["cpu_baseline"], "parity": r.get("parity")}
        if "h2d" in r:
            res["h2d"] = r["h2d"]
        if "note" in r:
            res["note"] = r["note"]
    hwm = peak_rss_gb()
    if hwm is not None:
        log(f"rank {rank}: peak host memory {hwm:.1f} GB")
    if rank == 0:
        if hwm is not None:
            res["host_peak_rss_gb"] = round(hwm, 2)      # this rank's VmHWM (the N=8 host-memory budget)
        if rehearsal:
            res["data"] = "rehearsal (GPUFLOW_BENCH_SELFTEST): the oracle stood in for the device; not a measurement"
        else:
            from cilium_amd import _lib
            res["build_id"] = _lib.BUILD_ID      # gf_build_id(): the sources libgpuflow.so was compiled from
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
