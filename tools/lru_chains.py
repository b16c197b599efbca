"""Per-event account of the LRU stand-in's launch chains in a rocprofv3 kernel
trace (tools/gpu.sh trace:...): one chain = one k_lru_chain launch (round 6), or the
first k_lru_sample .. k_lru_end (k_lru_round_end in round-5 traces).

    python tools/lru_chains.py gpurun_out/TAG/trace_NAME/run_kernel_trace.csv [--active-us 100]

Prints every chain that evicted (device time above --active-us) kernel by kernel,
then the count and mean time of the no-op chains (the count under the limit: the
sample kernel returns at once and the rest read the flag)."""
import argparse
import csv
import re


def name(k):
    return re.sub(r"^void ", "", k).split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--active-us", type=float, default=100.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    chains, cur = [], None
    for r in rows:
        n = name(r["Kernel_Name"])
        if n.startswith("k_lru_chain"):                 # round 6 on: the whole chain is one cooperative launch
            chains.append([(n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)])
            continue
        if n.startswith("k_lru_sample") and cur is None:
            cur = []
            chains.append(cur)
        if cur is not None and n.startswith("k_lru"):
            cur.append((n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
        if n.startswith("k_lru_round_end") or n.startswith("k_lru_end"):
            cur = None
    tot = lambda c: sum(d for _, d in c)
    act = [c for c in chains if tot(c) > a.active_us]
    idle = [tot(c) for c in chains if tot(c) <= a.active_us]
    print(f"{len(chains)} chains, {sum(map(tot, chains)) / 1e3:.3f} ms in all; {len(act)} evicted")
    for c in act:
        print(f"  {tot(c) / 1e3:.3f} ms: " + " ".join(f"{n.replace('k_lru_', '')}={d / 1e3:.3f}" for n, d in c))
    if idle:
        print(f"  no-op chains: {len(idle)}, mean {sum(idle) / len(idle):.1f} us")
    if act:
        print(f"  longest evicting chain {max(map(tot, act)) / 1e3:.3f} ms, mean {sum(map(tot, act)) / len(act) / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
