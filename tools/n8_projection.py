"""Wall-time projection of the driver's `bench.py --gpus 8` run from an N=1 run's
own phase times (its stderr log and JSON line) — the scaling run's per-rank work is
the N=1 work with L = W + K steps and no long horizon, and its parity sample is
bench.parity_div's (sized to the rank's share of the host's cores).

    python tools/n8_projection.py LOG JSON [--threads-per-rank T ...] > profiles/<tag>_n8_projection.json

Inputs read from the N=1 run: config 2's table and stream set-up times, the
oracle's parity throughput (packets compared / seconds, on `cores` threads), the
config-4 leg's wall time and its parity packets; every rank of the N=8 run does
the same set-up (the pair population is 8x larger: numpy work that scales with
it is scaled), runs its GPU legs (unchanged per rank: weak scaling), and checks
its own sample on T host threads.  The 8 ranks run concurrently, so the node's
wall time is one rank's (plus a contention factor, stated)."""
import argparse
import json
import math
import re
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("json")
    ap.add_argument("--threads-per-rank", type=int, nargs="+", default=[2, 4, 16])
    ap.add_argument("--contention", type=float, default=1.3,
                    help="slow-down of the host legs with 8 ranks on one host (memory bandwidth, not measured)")
    ap.add_argument("--startup-s", type=float, default=15.0, help="process start, torch import, HIP init")
    a = ap.parse_args()
    log = open(a.log).read()
    r = json.loads(open(a.json).read().strip().splitlines()[-1])
    t_tables = float(re.search(r"tables .* \(([\d.]+)s\)", log).group(1))
    t_gen = float(re.search(r"generated (\d+) steps \(([\d.]+)s\)", log).group(2))
    steps_gen = int(re.search(r"generated (\d+) steps", log).group(1))
    m = re.search(r"cpu baseline \+ parity: (\d+) packets compared.*on (\d+) threads \(([\d.]+)s\)", log)
    par_pk, par_thr, par_s = int(m.group(1)), int(m.group(2)), float(m.group(3)) - t_gen
    rate_thread = par_pk / par_s / par_thr               # packets / s / thread, compare included
    c4 = (r.get("configs") or {}).get("4") or {}
    m4 = re.search(r"config 4: [\d.]+ Mpps \(([\d.]+)s\)", log)
    t_c4 = float(m4.group(1)) if m4 else None
    c4_pk = (c4.get("parity") or {}).get("packets_compared")
    W, K = r["warmup"], r["steps"]
    W = max(W, 3)
    per_step = r["config"]["packets_per_step_per_gpu"]
    out = {"source_log": a.log, "source_json": a.json, "n1": {
        "tables_s": t_tables, "stream_s": t_gen, "stream_steps": steps_gen,
        "parity_packets": par_pk, "parity_s": round(par_s, 1), "parity_threads": par_thr,
        "oracle_packets_per_s_per_thread": round(rate_thread), "config4_s": t_c4, "config4_parity_packets": c4_pk},
        "assumptions": {"contention": a.contention, "startup_s": a.startup_s,
                        "pairs_scaling": "table set-up x 1.5 for the 8x pair population (numpy over 8M pairs)",
                        "config4": "per leg: the N=1 leg's time with its oracle part rescaled to the N=8 sample"},
        "projection": {}}
    L = W + K
    for T in a.threads_per_rank:
        args = argparse.Namespace(parity_div=0)
        div2 = bench.parity_div(args, 8, T, L * per_step)
        c2_oracle = L * per_step / div2 / (rate_thread * T)
        c2 = t_tables * 1.5 + t_gen * L / steps_gen + c2_oracle
        div4 = bench.parity_div(args, 8, T, 2 * (4 + max(4, K // 2)) * per_step) * 2
        c4_leg = None
        if t_c4 and c4_pk:
            c4_oracle_n1 = c4_pk / (rate_thread / 2 * par_thr)        # the pipeline oracle: ~half the rate
            c4_fixed = max(t_c4 - c4_oracle_n1, 0.0)
            c4_pk8 = (4 + max(4, K // 2)) * per_step / div4
            c4_leg = c4_fixed + c4_pk8 / (rate_thread / 2 * T)
        legs = {"config2_s": round(c2, 1), "config2_parity_div": div2, "config4_owned_s": c4_leg and round(c4_leg, 1),
                "config4_exchange_s": c4_leg and round(c4_leg * 1.1, 1), "config4_parity_div": div4}
        total = a.startup_s + (c2 + (2.1 * c4_leg if c4_leg else 0.0)) * a.contention
        out["projection"][f"T{T}"] = dict(legs, total_s=round(total, 1), within_390s=total <= 390)
    rss = r.get("host_peak_rss_gb")
    if rss:
        # every rank holds what the N=1 run held at its peak, less the part of its oracle
        # sample the larger parity divisor removes (not modelled: an upper bound)
        out["host_memory"] = {"n1_peak_rss_gb": rss, "node_upper_bound_gb": round(8 * rss, 1),
                              "note": "8 ranks x the N=1 peak; each rank's parity sample is smaller at N=8"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
