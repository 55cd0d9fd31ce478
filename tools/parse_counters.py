"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch) -> OUT/summary.json, and
write profiles/traffic_latest.json (HBM bytes per launch of each kernel, gfx950-corrected:
FETCH_SIZE x 2 per MI355X_MICROARCH.md §HBM, + WRITE_SIZE; both in KiB)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    out = Path(sys.argv[1])
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(out.glob("p*/**/*counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            name = r.get("Kernel_Name", "")
            short = name.split("(")[0].replace("slamhot::", "")
            acc[short][r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    summary = {}
    for k, cs in acc.items():
        d = {}
        for c, vals in cs.items():
            per = defaultdict(float)
            for disp, v in vals:
                per[disp] += v
            d[c] = sum(per.values()) / max(len(per), 1)
        summary[k] = d
    (out / "summary.json").write_text(json.dumps(summary, indent=1, sort_keys=True))
    traffic = {}
    for k, d in summary.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            traffic[k] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    for k, d in sorted(summary.items()):
        print(k, {c: round(v, 1) for c, v in sorted(d.items())})
    print("traffic bytes/launch:", {k: int(v) for k, v in traffic.items()})
    (out / "traffic.json").write_text(json.dumps(traffic, indent=1))
    if len(sys.argv) > 2 and sys.argv[2] in traffic:
        # bench.py reads this for roofline.traffic: kernel, shape of the run, HBM bytes / launch
        k = sys.argv[2]
        meta = dict(kernel=k, batch=int(sys.argv[3]), width=int(sys.argv[4]), bytes_per_launch=int(traffic[k]),
                    fetch_size_kib=summary[k]["FETCH_SIZE"], write_size_kib=summary[k]["WRITE_SIZE"],
                    note="2 x FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md HBM section (the x2 is calibrated "
                         "there for 16 B/lane streaming reads; this kernel stages with 4 B/lane loads)")
        Path("profiles/traffic_latest.json").write_text(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
