#!/bin/bash
# LBA leg value vs calls per solver (ramp-up / tail amortisation), interleaved.
export TMPDIR=/tmp
for i in 1 2 3; do
  for c in "$@"; do
    timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline --lba-calls $c > gpurun_out/lbac.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lbac.json'))['lba']; print('calls=$c', d['value'], d['ms_per_call'], d['host_plan_ms_per_call'])"
  done
done
