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
    # FETCH_SIZE -> bytes: the factor measured by tools/microbench/mb_fetch for the load width
    # the kernel stages with (profiles/fetch_calibration.json; 2.0 = the guide's 16 B/lane value)
    fac = {"k_fast_wave": "4"}
    cal = {}
    cf = Path("profiles/fetch_calibration.json")
    if cf.exists():
        cal = json.loads(cf.read_text()).get("factor_by_lane_bytes", {})
    traffic = {}
    for k, d in summary.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            f = float(cal.get(fac.get(k, "16"), 2.0))
            traffic[k] = (f * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    for k, d in sorted(summary.items()):
        print(k, {c: round(v, 1) for c, v in sorted(d.items())})
    print("traffic bytes/launch:", {k: int(v) for k, v in traffic.items()})
    (out / "traffic.json").write_text(json.dumps(traffic, indent=1))
    if len(sys.argv) > 2 and sys.argv[2] in traffic:
        # bench.py reads this for roofline.traffic: kernel, shape of the run, HBM bytes / launch
        k = sys.argv[2]
        f = float(cal.get(fac.get(k, "16"), 2.0))
        d = summary[k]
        # dispatches of the kernel per batch (k_fast_wave: one per cell class):
        # the per-dispatch means times this are the batch's figures, what bench.py's roofline uses
        nd = int(sys.argv[5]) if len(sys.argv) > 5 else 1
        meta = dict(kernel=k, batch=int(sys.argv[3]), width=int(sys.argv[4]), dispatches_per_batch=nd,
                    bytes_per_launch=int(nd * traffic[k]),
                    fetch_size_kib=nd * d["FETCH_SIZE"], write_size_kib=nd * d["WRITE_SIZE"], fetch_factor=f,
                    valu_instr_per_launch=nd * d["SQ_INSTS_VALU"] if d.get("SQ_INSTS_VALU") else None,
                    lds_bank_conflict_per_lds_active=(d["SQ_LDS_BANK_CONFLICT"] / d["SQ_ACTIVE_INST_LDS"]
                                                      if d.get("SQ_ACTIVE_INST_LDS") else None),
                    note=f"({f:g} x FETCH_SIZE + WRITE_SIZE) x {nd} dispatches per batch; the FETCH_SIZE factor is measured for this kernel's "
                         f"{fac.get(k, '16')} B/lane loads by tools/microbench/mb_fetch (profiles/fetch_calibration.json)")
        Path("profiles/traffic_latest.json").write_text(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
