"""Per-step time of the gpuflow kernels from a rocprofv3 kernel_stats.csv
(rocPRIM kernels of libgpuflow are the ROCPRIM_400200 namespace; 400001 is
torch's own rocPRIM, used by the bench's stream generator)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
for r in csv.DictReader(open(path)):
    n = r["Name"]
    if "k_" in n.split("(")[0] or "ROCPRIM_400200" in n:
        short = n.split("(")[0].replace("void ", "")
        if "rocprim" in short:
            short = "rocprim::" + short.split("::")[-1][:40]
        print(f"{short[:60]:60s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs']) / 1e6:8.4f} "
              f"ms/step={float(r['TotalDurationNs']) / 1e6 / steps:8.4f}")
