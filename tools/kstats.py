"""Print per-step time of the gpuflow kernels from a rocprofv3 kernel_stats.csv."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0   # bench: warmup 3 + steps 4 launches
for r in csv.DictReader(open(path)):
    if r["Name"].startswith("k_") or "rocprim" in r["Name"]:
        print(f"{r['Name'][:40]:40s} calls={r['Calls']:>5s} ms/step={float(r['TotalDurationNs']) / 1e6 / steps:8.3f}")
