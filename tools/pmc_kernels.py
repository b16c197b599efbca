"""Per-kernel PMC summary of one bench configuration: every counter of every
rocprofv3 --pmc pass under DIR (DIR/p*/run_counter_collection.csv, one counter
group per pass, tools/profile_round.sh), summed per kernel over the classify
calls of the run and divided by the bench steps the process ran (warm-up +
timed), so each number is "per step".

Derived per kernel:
  traffic_bytes      the L2 -> fabric bytes, from the request-size counters when
                     the run has them (round 4 on): reads = 128 x RDREQ_128B + 32 x
                     RDREQ_32B + 64 x the rest, writes = 64 x WRREQ_64B + 32 x the
                     rest.  On gfx950 FETCH_SIZE prices a 128-B read request at 64 B
                     (it counts TCC_BUBBLE, which stays 0 there), so it reports half
                     of every line fill: random 16-B loads are 128-B requests
                     (profiles/r4_primbench_pmc.txt).  Runs without those counters
                     fall back to FETCH_SIZE + WRITE_SIZE (KB in the CSV) x 1024,
                     uncorrected, and say so ("traffic_model").
  reads / writes     per packet: 128-B line reads, partial (32-B) writes, full
                     64-B writes, atomics (counted among the writes)
  l2_hit_rate        TCC_HIT / (TCC_HIT + TCC_MISS)
  ea_requests        TCC_EA0_RDREQ_sum + TCC_EA0_WRREQ_sum (L2 -> fabric requests)
  wave_insts         SQ_INSTS_VALU + SQ_INSTS_SALU (wave-instructions)
  GRBM_GUI_ACTIVE    kept raw: / 8 XCDs / the kernel's time = its effective clock
                     (bench.py divides by the live launch time)

  python tools/pmc_kernels.py DIR --bench-json DIR/p1.json --out profiles/<tag>_pmc_kernels_c<cfg>.json
"""
import argparse
import collections
import csv
import glob
import json
import re
import os

STEP_ENTRY = {"k_pipe_front", "k_eg_front", "k_ing_pack", "k_xdp", "k_xdp_lds", "k_lb", "k_parse"}


def short(name):
    s = name.split("(")[0].replace("void ", "").strip()
    if "rocprim" in s or "ROCPRIM" in name:
        return "rocprim"
    if s.startswith("k_ing_groups") or s.startswith("k_eg_"):
        # the family template argument names the kernel (k_ing_groups / k_ing_groups6);
        # a second one (k_ing_groups' queue grab) does not; of the flags after it, the
        # first (per-endpoint CT maps) names the _pct instances, the second (the egress
        # related-entry set) does not
        s = re.sub(r"<([46])(, *\d+)?(, *(true|false))?(, *(true|false))?>",
                   lambda m: ("6" if m.group(1) == "6" else "") + ("_pct" if m.group(4) == "true" else ""), s)
    return s


def per_kernel(path, nsteps):
    rows = list(csv.DictReader(open(path)))
    base = lambda n: n.split("(")[0].replace("void ", "").split("<")[0].strip()
    first = min((int(r["Dispatch_Id"]) for r in rows if base(r["Kernel_Name"]) in STEP_ENTRY), default=0)
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d < first:
            continue
        k = short(r["Kernel_Name"])
        out[k][r["Counter_Name"]] += float(r["Counter_Value"]) / nsteps
        disp[k].add(d)
    return out, {k: len(v) / nsteps for k, v in disp.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bench-json", required=True, help="the bench line of one pass (steps, warmup, packets)")
    ap.add_argument("--packets", type=int, default=0, help="packets per step (default: from the bench line)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernel-stats", default="", help="rocprofv3 --stats CSV of the same configuration: each "
                    "kernel's average duration goes into the summary (bench.py's roofline.frac_rocprof)")
    a = ap.parse_args()
    b = json.loads(open(a.bench_json).read().strip().splitlines()[-1])
    nsteps = int(b["steps"]) + int(b["warmup"])
    cf = b.get("config", {})
    pk = a.packets or int(b.get("packets_per_step") or cf.get("packets_per_step_per_gpu") or cf.get("packets_per_step") or 0)
    ks = collections.defaultdict(dict)
    dps = {}
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "run_counter_collection.csv"))):
        c, d = per_kernel(f, nsteps)
        for k, v in c.items():
            ks[k].update(v)
        dps.update(d)
    res = {"packets_per_step": pk, "steps_run": nsteps, "source": os.path.relpath(a.dir),
           "build_id": b.get("build_id"), "kernels": {}}
    for k, c in sorted(ks.items()):
        e = {"dispatches_per_step": round(dps.get(k, 0), 3), "counters_per_step": {n: round(v, 1) for n, v in sorted(c.items())}}
        if "TCC_EA0_RDREQ_128B_sum" in c and "TCC_EA0_WRREQ_64B_sum" in c:
            rd, r128, r32 = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_RDREQ_128B_sum"], c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            wr, w64, at = c.get("TCC_EA0_WRREQ_sum", 0.0), c["TCC_EA0_WRREQ_64B_sum"], c.get("TCC_EA0_ATOMIC_sum", 0.0)
            rb = 128 * r128 + 32 * r32 + 64 * max(rd - r128 - r32, 0.0)
            wb = 64 * w64 + 32 * max(wr - w64, 0.0)
            e["traffic_model"] = "request sizes (128-B line reads, 32/64-B writes)"
            e["read_bytes"], e["write_bytes"] = rb, wb
            e["traffic_bytes"] = rb + wb
            e["traffic_bytes_per_packet"] = (rb + wb) / pk if pk else None
            if pk:
                e["per_packet"] = {"line_reads": round(rd / pk, 4), "reads_128B": round(r128 / pk, 4),
                                   "partial_writes": round(max(wr - w64 - at, 0.0) / pk, 4),
                                   "full_writes_64B": round(w64 / pk, 4), "atomics": round(at / pk, 4)}
        elif "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            t = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024
            e["traffic_model"] = "FETCH_SIZE + WRITE_SIZE (uncorrected)"
            e["traffic_bytes"] = t
            e["traffic_bytes_per_packet"] = t / pk if pk else None
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        if "TCC_EA0_RDREQ_sum" in c:
            e["ea_requests"] = c["TCC_EA0_RDREQ_sum"] + c.get("TCC_EA0_WRREQ_sum", 0.0)
            e["ea_requests_per_packet"] = e["ea_requests"] / pk if pk else None
        if "SQ_INSTS_VALU" in c:
            e["wave_insts"] = c["SQ_INSTS_VALU"] + c.get("SQ_INSTS_SALU", 0.0)
            e["wave_insts_per_64_packets"] = e["wave_insts"] * 64 / pk if pk else None
        res["kernels"][k] = e
    if a.kernel_stats:
        res["kernel_stats_source"] = os.path.relpath(a.kernel_stats)
        tot = collections.defaultdict(lambda: [0, 0.0])
        for r in csv.DictReader(open(a.kernel_stats)):
            k = short(r["Name"])
            tot[k][0] += int(r["Calls"])
            tot[k][1] += float(r["TotalDurationNs"])
        for k, (n, t) in tot.items():
            if k in res["kernels"] and n:
                res["kernels"][k]["rocprof_calls"] = n
                res["kernels"][k]["rocprof_avg_ns"] = round(t / n, 1)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: {x: y for x, y in v.items() if x != "counters_per_step"} for k, v in res["kernels"].items()},
                     indent=1))


if __name__ == "__main__":
    main()
