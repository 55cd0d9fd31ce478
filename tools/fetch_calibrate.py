"""FETCH_SIZE calibration from `rocprofv3 --pmc FETCH_SIZE -- tools/microbench/mb_fetch`:
bytes read per launch (1 GiB) / (FETCH_SIZE KiB x 1024) per load width ->
profiles/fetch_calibration.json {factor_by_lane_bytes: {"4": f4, "8": f8, "16": f16}}."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

BYTES = 1 << 30


def main():
    out = Path(sys.argv[1])
    per = defaultdict(lambda: defaultdict(float))
    for f in sorted(out.glob("**/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "k_read" not in name:
                continue
            w = "16" if "unsigned int, 4u" in name else "8" if "unsigned int, 2u" in name else "4"
            per[w][int(r.get("Dispatch_Id", 0))] += float(r["Counter_Value"])
    res = {}
    for w, disp in per.items():
        vals = sorted(disp.values())
        med = vals[len(vals) // 2]
        res[w] = {"fetch_size_kib_median": med, "launches": len(vals), "factor": BYTES / (med * 1024.0)}
    cal = {"bytes_per_launch": BYTES, "per_width": res,
           "factor_by_lane_bytes": {w: round(v["factor"], 4) for w, v in res.items()},
           "source": "tools/microbench/mb_fetch.hip under rocprofv3 --pmc FETCH_SIZE"}
    Path("profiles/fetch_calibration.json").write_text(json.dumps(cal, indent=1))
    print(json.dumps(cal))


if __name__ == "__main__":
    main()
