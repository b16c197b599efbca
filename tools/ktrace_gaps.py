"""Idle gaps of the GPU between consecutive kernels of a rocprofv3 --kernel-trace
CSV (run_kernel_trace.csv): per step, the time no kernel ran, and the kernels the
largest gaps follow / precede (host round trips: syncs, readbacks, launch work).
  python tools/ktrace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [--top 15]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--dump", type=int, default=-1, help="list the dispatches of this step (0-based) with the gap before each")
    ap.add_argument("--entry", required=True, help="the step's first kernel (e.g. k_eg_front): analysis starts at its "
                                                   "first dispatch; totals are divided by its dispatch count")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    short = lambda n: n.split("(")[0].replace("void ", "")[:48]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    first = next(i for i, k in enumerate(ks) if a.entry in k[2])
    ks = ks[first:]
    steps = sum(1 for k in ks if k[2].startswith(a.entry))
    if a.dump >= 0:
        st = [i for i, k in enumerate(ks) if k[2].startswith(a.entry)]
        lo, hi = st[a.dump], st[a.dump + 1] if a.dump + 1 < len(st) else len(ks)
        for i in range(lo, hi):
            g = (ks[i][0] - ks[i - 1][1]) / 1e3 if i else 0.0
            print(f"  gap {g:8.1f} us  run {(ks[i][1] - ks[i][0]) / 1e3:8.1f} us  {ks[i][2]}")
    gaps = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    end = ks[0][1]
    for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
        busy += (e0 - s0) / 1e6
        g = (s1 - max(end, e0)) / 1e6
        end = max(end, e0)
        if 0.005 < g < 1.0:                              # (longer: outside the steps)
            gaps[(n0, n1)][0] += 1
            gaps[(n0, n1)][1] += g
    span = (ks[-1][1] - ks[0][0]) / 1e6
    print(f"{steps} steps from the first {a.entry}: dispatches {len(ks)}  span {span:.3f} ms  kernel time {busy:.3f} ms  "
          f"idle {span - busy:.3f} ms  (per step: span {span / steps:.3f}, idle {(span - busy) / steps:.3f})")
    for (n0, n1), (c, g) in sorted(gaps.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{g / steps:9.4f} ms/step in {c / steps:6.1f} gaps/step  after {n0:48s} before {n1}")


if __name__ == "__main__":
    main()
