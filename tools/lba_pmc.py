"""profiles/<tag>_lba_pmc.json from the LBA PMC pass (tools/round_evidence.sh step 4):
executed FP64 FLOP per launch = (2 FMA + ADD + MUL) x 64 + MFMA_MOPS x 512 (counter_defs.yaml
TOTAL_64_OPS form), MFMA busy cycles and GRBM_GUI_ACTIVE per kernel."""
import json
import sys
from pathlib import Path

src, tag = Path(sys.argv[1]), sys.argv[2]
s = json.loads((src / "summary.json").read_text())
out = {"source": "rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 "
                 "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 bench.py "
                 "--legs lba --no-cpu-baseline --lba-calls 1 (tools/round_evidence.sh)",
       "flop": "TOTAL_64_OPS = (2 FMA + ADD + MUL) x 64 + MFMA_MOPS x 512 per launch",
       "time_us": "GRBM_GUI_ACTIVE / 8 XCDs / 2.1 GHz (approximate: profiled clocks run below nominal)",
       "kernels": {}}
for k, d in sorted(s.items()):
    if "lba::" not in k:
        continue
    v = 64 * (2 * d.get("SQ_INSTS_VALU_FMA_F64", 0) + d.get("SQ_INSTS_VALU_ADD_F64", 0) + d.get("SQ_INSTS_VALU_MUL_F64", 0))
    m = 512 * d.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
    out["kernels"][k] = {"fp64_flop_per_launch": round(v + m), "mfma_f64_flop_per_launch": round(m),
                         "SQ_VALU_MFMA_BUSY_CYCLES": d.get("SQ_VALU_MFMA_BUSY_CYCLES"),
                         "GRBM_GUI_ACTIVE": d.get("GRBM_GUI_ACTIVE"),
                         "time_us": round(d.get("GRBM_GUI_ACTIVE", 0) / 8 / 2.1e3, 1)}
Path(f"profiles/{tag}_lba_pmc.json").write_text(json.dumps(out, indent=1))
for k, v in out["kernels"].items():
    print(f"{k:28s} {v['time_us']:8.1f} us {v['fp64_flop_per_launch'] / 1e6:9.1f} MFLOP")
