"""GPU-busy fraction from a rocprofv3 --kernel-trace CSV directory: union of kernel intervals
over the span of the named kernels' launches, plus per-kernel totals inside that span."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "lba::"
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
sel = [r for r in rows if pat in r[2]]
t0, t1 = min(r[0] for r in sel), max(r[1] for r in sel)
iv = sorted((s, e) for s, e, _ in rows if e > t0 and s < t1)
busy, cs, ce = 0, None, None
for s, e in iv:
    s, e = max(s, t0), min(e, t1)
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"span {(t1 - t0) / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({100 * busy / (t1 - t0):.1f}%)")
agg = defaultdict(lambda: [0, 0])
for s, e, n in rows:
    if e > t0 and s < t1:
        agg[n][0] += 1
        agg[n][1] += e - s
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:16]:
    print(f"{n[-40:]:40s} n={c:6d} sum={t / 1e6:8.2f} ms avg={t / c / 1e3:8.1f} us")
