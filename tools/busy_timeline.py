"""GPU busy fraction (union of kernel intervals) per time bucket of a rocprofv3 kernel trace, with
the kernels that start in each bucket.  Usage: busy_timeline.py TRACE.csv [bucket_ms] [nbuckets]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
bucket = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 5e6
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 40
name = lambda s: (re.findall(r"(k_\w+|__amd_\w+)", s) or [s[:20]])[0]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r["Kernel_Name"])) for r in rows)
t0 = iv[0][0]


def busy(a, b):
    tot, cs, ce = 0, None, None
    for s, e, _ in iv:
        if e < a or s > b:
            continue
        s, e = max(s, a), min(e, b)
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


for k in range(nb):
    a = t0 + k * bucket
    ks = [n for s, e, n in iv if a <= s < a + bucket]
    top = sorted(set(ks), key=lambda n: -ks.count(n))[:5]
    print(f"{k * bucket / 1e6:8.1f} ms busy {busy(a, a + bucket) / bucket:5.3f} kernels {len(ks):5d} {top}")
