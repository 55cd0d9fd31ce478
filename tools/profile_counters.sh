#!/bin/bash
# Collect per-kernel PMC counters for bench.py on the GPU box (one rocprofv3 pass per group;
# --pmc is never combined with trace domains).  Usage: tools/profile_counters.sh OUTDIR [bench args]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" \
  "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
done
python3 tools/parse_counters.py "$OUT"
