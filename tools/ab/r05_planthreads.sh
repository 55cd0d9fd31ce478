#!/bin/bash
# LBA leg (bench.py --legs lba) per planning-thread cap (SLAMHOT_LBA_PLAN_THREADS), interleaved x3.
# Usage: r05_planthreads.sh "4 6 8"
export TMPDIR=/tmp
for i in 1 2 3; do
  for t in ${1:-4 6 8}; do
    SLAMHOT_LBA_PLAN_THREADS=$t timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline > gpurun_out/planthr.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/planthr.json'))['lba']
print('threads $t', 'LM it/s', d['value'], 'plan ms/call', d['host_plan_ms_per_call'], 'ms/call', d['ms_per_call'])"
  done
done
