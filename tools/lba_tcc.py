"""L2 behaviour per LBA kernel from one rocprofv3 --pmc pass (TCC_HIT_sum, TCC_MISS_sum,
TCC_EA0_RDREQ_sum): hit rate, memory-side read requests and the FETCH_SIZE-equivalent bytes per
launch (RDREQ x 64 B, doubled for gfx950's 128-B requests tallied at 64 B: MI355X_MICROARCH.md,
HBM section; Infinity-Cache hits are counted too, so this bounds HBM reads from above).
usage: python tools/lba_tcc.py PMC_DIR [OUT.json]"""
import collections
import csv
import json
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    f = next(d.rglob("*counter_collection.csv"))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("::")[-1]
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    out = {"source": f"rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE over {f.name}",
           "bytes_rule": "memory-side read bytes per launch = TCC_EA0_RDREQ_sum x 64 B x 2 (gfx950 128-B requests "
                         "tallied at 64 B); Infinity-Cache hits included",
           "kernels": {}}
    for k, c in sorted(per.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        n = len(disp[k])
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        out["kernels"][k] = {
            "launches": n,
            "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
            "l2_requests_per_launch": round((hit + miss) / n),
            "mem_read_MB_per_launch": round(c.get("TCC_EA0_RDREQ_sum", 0) * 128 / n / 1e6, 3),
            "GRBM_GUI_ACTIVE_per_launch": round(c.get("GRBM_GUI_ACTIVE", 0) / n),
        }
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
