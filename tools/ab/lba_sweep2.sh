#!/bin/bash
# LBA leg: solvers in flight with and without the GPU phase lock (SLAMHOT_LBA_EXCLUSIVE)
export TMPDIR=/tmp
for ex in 0 1; do
for cfg in "128 2" "128 3" "128 4" "256 2" "256 3"; do
  set -- $cfg
  SLAMHOT_LBA_EXCLUSIVE=$ex timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline --lba-windows $1 --lba-inflight $2 --lba-calls 6 > gpurun_out/lbasw_$1_$2_$ex.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/lbasw_$1_$2_$ex.json'))['lba']; print('ex=$ex $1 x $2', d['value'], d['roofline']['frac'], d['host_plan_ms_per_call'])"
done
done
