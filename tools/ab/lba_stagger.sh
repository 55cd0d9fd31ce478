#!/bin/bash
# LBA leg: solver start stagger / calls / solvers scan (whole-job LM iterations/s)
export TMPDIR=/tmp
for cfg in "4 6 5" "4 6 3" "4 6 7" "4 8 5" "5 6 4" "6 6 3" "4 6 5"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline --lba-inflight $1 --lba-calls $2 --lba-stagger-ms $3 > gpurun_out/stg.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/stg.json'))['lba']; print('inflight=$1 calls=$2 stagger=$3', d['value'], d['ms_per_call'], d['host_plan_ms_per_call'])"
done
