#!/bin/bash
# LBA leg vs planning threads per call (SLAMHOT_LBA_PLAN_THREADS), interleaved; one timing print.
export TMPDIR=/tmp
SLAMHOT_LBA_PLAN_TIMING=1 timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline --lba-calls 2 2>&1 >/dev/null | grep "lba plan" | tail -4
for i in 1 2 3; do
  for t in "$@"; do
    SLAMHOT_LBA_PLAN_THREADS=$t timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline > gpurun_out/lbap.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lbap.json'))['lba']; print('threads=$t', d['value'], d['ms_per_call'], d['host_plan_ms_per_call'])"
  done
done
