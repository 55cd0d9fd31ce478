#!/bin/bash
# LBA leg: windows per call x solvers in flight x start stagger (whole-job LM iterations/s)
export TMPDIR=/tmp
for cfg in "128 4 6" "64 4 3" "64 6 3" "64 8 2" "96 4 5" "32 8 1.5" "128 4 6"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline --lba-windows $1 --lba-inflight $2 --lba-stagger-ms $3 > gpurun_out/lbaw.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/lbaw.json'))['lba']; print('windows=$1 inflight=$2 stagger=$3', d['value'], d['ms_per_call'], d['host_plan_ms_per_call'])"
done
