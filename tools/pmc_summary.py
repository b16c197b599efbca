"""Summarise rocprofv3 --pmc passes over bench.py (tools/profile_round.sh) into
per-launch numbers for the dominant kernel, k_ing_groups.

Steady-state launches only: the bench's first W launches run on a stream that
is still filling (1/4, 2/4, 3/4 of the flows), so the last `--steps` launches
of each pass are averaged.

Byte counters (KB in rocprofv3's CSV):
  * FETCH_SIZE = 64 B per memory-side read request (TCC_EA0_RDREQ x 64 B).
    The MI355X guide's 2x correction is for wide streaming reads; every read
    of this kernel is a random 16-32 B access, for which tools/primbench.hip
    calibrates FETCH_SIZE at exactly one 64-B request per load
    (profiles/r1_pmc_calibration.json), so FETCH_SIZE is used as is.
  * WRITE_SIZE = 32 B per write request / atomic (same calibration).
"""
import argparse
import collections
import csv
import glob
import json
import os

KERNEL = "k_ing_groups"
STEP_ENTRY = {"k_pipe_front", "k_eg_front", "k_ing_pack", "k_xdp", "k_xdp_lds", "k_lb", "k_parse"}


def per_launch(path, nsteps):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        name = r["Kernel_Name"]
        if KERNEL in name and "ILi6E" not in name and "<6>" not in name:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ds = sorted(per)[-nsteps:]
    out = collections.defaultdict(float)
    for d in ds:
        for c, v in per[d].items():
            out[c] += v / len(ds)
    return out


def per_step(path, names, nsteps):
    """Counters summed over every dispatch of the kernels matching `names`
    (substrings; "gpuflow" = every libgpuflow kernel: k_* and its rocPRIM
    instantiations), divided by the number of bench steps the process ran."""
    out = collections.defaultdict(float)
    rows = list(csv.DictReader(open(path)))
    # the classify calls only: from the first dispatch of a step's entry kernel on
    # (the tables' setup before it — bulk inserts of pre-filled CT maps, pushes —
    # is not part of any step)
    first = min((int(r["Dispatch_Id"]) for r in rows
                 if r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0] in STEP_ENTRY), default=0)
    for r in rows:
        if int(r["Dispatch_Id"]) < first:
            continue
        name = r["Kernel_Name"]
        short = name.split("(")[0]
        ok = any((n == "gpuflow" and (" k_" in " " + short.replace("void ", "") or "ROCPRIM_400200" in name))
                 or (n != "gpuflow" and n in short) for n in names)
        if ok:
            out[r["Counter_Name"]] += float(r["Counter_Value"]) / nsteps
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--packets", type=int, default=16777216, help="packets per launch (bench config 2)")
    ap.add_argument("--kernels", default=None,
                    help="per-step mode: comma list of kernel-name substrings summed over all their dispatches")
    ap.add_argument("--nsteps", type=int, default=0, help="per-step mode: bench steps run (warm-up + timed)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    global KERNEL
    c = {}
    for f in glob.glob(os.path.join(a.dir, "*", "run_counter_collection.csv")):
        if a.kernels:
            c.update(per_step(f, a.kernels.split(","), a.nsteps))
        else:
            c.update(per_launch(f, a.steps))
    if a.kernels:
        KERNEL = a.kernels
    n = a.packets
    fetch = c.get("FETCH_SIZE", 0.0) * 1024
    write = c.get("WRITE_SIZE", 0.0) * 1024
    hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
    res = {
        "kernel": KERNEL,
        "packets_per_launch": n,
        "launches_averaged": a.steps,
        "counters_per_launch": {k: round(v, 1) for k, v in sorted(c.items())},
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "traffic_bytes_per_launch": fetch + write,
        "traffic_bytes_per_packet": (fetch + write) / n,
        "ea_requests_per_packet": {
            "read": c.get("TCC_EA0_RDREQ_sum", 0.0) / n,
            "write_incl_atomics": c.get("TCC_EA0_WRREQ_sum", 0.0) / n,
            "atomic": c.get("TCC_EA0_ATOMIC_sum", 0.0) / n,
        },
        "l2_hit_rate": hit / (hit + miss) if hit is not None and miss else None,
        "calibration": "FETCH_SIZE used raw: random 16-32 B loads are one 64-B request each "
                       "(tools/primbench.hip under --pmc; profiles/r1_pmc_calibration.json)",
    }
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main()
