#!/bin/bash
# The LBA leg alone vs after the headline + extract legs in one bench process (interleaved x2):
# does the state the earlier legs leave move the bench line's LBA number?
export TMPDIR=/tmp
for i in 1 2; do
  for legs in lba headline,extract,lba; do
    timeout -k 10 400 python bench.py --legs $legs --no-cpu-baseline > gpurun_out/lbaorder.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/lbaorder.json')); l=d['lba']
print('$legs', 'lba', l['value'], 'plan', l['host_plan_ms_per_call'], 'ms/call', l['ms_per_call'], 'dev 1 solver', l['device_lm_iters_per_s_one_solver'])"
  done
done
