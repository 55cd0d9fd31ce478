"""Per-kernel, per-grid-size average durations from a rocprofv3 --kernel-trace CSV directory."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
agg = defaultdict(list)
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = (name.split("(")[0][-40:], r.get("Grid_Size_X") or r.get("Grid_Size", ""))
        agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (k, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:42s} grid={g:>9s} n={len(v):4d} avg={sum(v)/len(v)/1e3:9.1f}us tot={sum(v)/1e6:8.2f}ms")
