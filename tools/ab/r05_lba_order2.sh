#!/bin/bash
# Which earlier leg slows the LBA leg (bench.py --legs X,lba), with the GPU clock / power sampled
# by rocm-smi right before and after each run.
export TMPDIR=/tmp
for legs in extract,lba pose,lba lba; do
  timeout -k 10 60 rocm-smi --showpower --showtemp --showsclk 2>/dev/null | grep -E "Socket|Temperature|sclk|Power" | head -6 | tr '\n' ' '; echo
  timeout -k 10 400 python bench.py --legs $legs --no-cpu-baseline > gpurun_out/lbaorder2.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/lbaorder2.json')); l=d['lba']
print('$legs', 'lba', l['value'], 'plan', l['host_plan_ms_per_call'], 'ms/call', l['ms_per_call'])"
done
timeout -k 10 60 rocm-smi --showpower --showtemp --showsclk 2>/dev/null | grep -E "Socket|Temperature|sclk|Power" | head -6 | tr '\n' ' '; echo
