"""Per-test request counters of the primbench matrix (tools/primbench.hip matrix
under rocprofv3 --pmc, one counter group per pass: tools/gpu_r4a.sh), normalised
per access (16.8M accesses per launch, the mean of each test's 3 launches).

  python tools/prim_pmc.py gpurun_out/r4a/prim > profiles/r4_primbench_pmc.txt
"""
import collections
import csv
import glob
import os
import sys

ACC = 1 << 24
COLS = [("TCC_EA0_RDREQ_sum", "rd"), ("TCC_EA0_RDREQ_128B_sum", "rd128"), ("TCC_EA0_RDREQ_32B_sum", "rd32"),
        ("TCC_EA0_WRREQ_sum", "wr"), ("TCC_EA0_WRREQ_64B_sum", "wr64"), ("TCC_EA0_ATOMIC_sum", "atom"),
        ("TCC_HIT_sum", "hit"), ("TCC_MISS_sum", "miss"), ("TCC_EA0_RDREQ_DRAM_sum", "rdDRAM"),
        ("TCC_EA0_WRREQ_DRAM_sum", "wrDRAM"), ("TCC_EA0_RDREQ_LEVEL_sum", "rdLevel"),
        ("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "stall"), ("FETCH_SIZE", "FETCH_KB"), ("WRITE_SIZE", "WRITE_KB")]


def tests():
    """The launch order of primbench's matrix (3 launches each)."""
    t = []
    for fp in ["128MB", "2GB", "16GB"]:
        t += [f"rd W={w} L={l} {fp}" for w, l in [(16, 1), (16, 2), (16, 4), (16, 8), (64, 1), (64, 2), (64, 4),
                                                   (128, 1), (128, 2)]]
    for fp in ["2GB", "16GB"]:
        t += [f"chain L={l} WPS={w} {fp}" for w in [1, 2, 4, 8] for l in [1, 2, 4]]
    t += [f"chain+2st L={l} WPS={w} 16GB" for w in [2, 4, 8] for l in [1, 2]]
    for fp in ["128MB", "2GB", "16GB"]:
        t += [f"st W={w} {fp}" for w in [4, 8, 16, 32, 64, 128]]
    for fp in ["128MB", "2GB", "16GB"]:
        t += [f"atomic u64 x{k} {fp}" for k in [1, 2]]
    for fp in ["128MB", "2GB", "16GB"]:
        t += [f"mix rd+st {fp}", f"rmw rd+8B st {fp}"]
    return t + ["seq read 4GB (per 256 B)", "seq write 4GB (per 256 B)"]


def main(d):
    data, names = collections.defaultdict(dict), {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            names[k] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            data[k][r["Counter_Name"]] = float(r["Counter_Value"])
    ds = sorted(k for k in names if not names[k].startswith("__amd"))
    groups, i = [], 0
    while i < len(ds):
        g = [ds[i]]
        i += 1
        while i < len(ds) and names[ds[i]] == names[g[0]] and len(g) < 3:
            g.append(ds[i])
            i += 1
        groups.append(g)
    print("# per access (primbench matrix, tools/gpu_r4a.sh); rd* = L2->fabric read requests by size, wr* = write")
    print("# requests (atomics are among them), hit/miss = L2 tag lookups, rdLevel = read requests in flight summed")
    print("# per cycle / requests (latency proxy, not normalised), FETCH/WRITE_KB = rocprof's derived sizes")
    print("%-28s" % "test" + "".join("%9s" % s for _, s in COLS) + "  kernel")
    for t, g in zip(tests(), groups):
        av = {c: sum(data[k].get(c, 0.0) for k in g) / len(g) for c, _ in COLS}
        row = []
        for c, s in COLS:
            v = av[c] / ACC
            row.append("%9.0f" % (av[c] / max(av["TCC_EA0_RDREQ_sum"], 1.0)) if s == "rdLevel" else "%9.3f" % v)
        print("%-28s" % t + "".join(row) + "  " + names[g[0]])


if __name__ == "__main__":
    main(sys.argv[1])
