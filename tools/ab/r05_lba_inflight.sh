#!/bin/bash
# LBA leg after the headline + extract legs (the default bench order) per solvers in flight.
# Usage: r05_lba_inflight.sh "3 4 5"
export TMPDIR=/tmp
for i in 1 2; do
  for n in ${1:-3 4 5}; do
    timeout -k 10 400 python bench.py --legs headline,extract,lba --lba-inflight $n --no-cpu-baseline > gpurun_out/lbainf.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/lbainf.json')); l=d['lba']
print('inflight $n', 'lba', l['value'], 'plan', l['host_plan_ms_per_call'], 'ms/call', l['ms_per_call'], 'headline', d['value'])"
  done
done
