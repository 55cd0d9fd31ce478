#!/bin/bash
# LBA leg throughput over (windows per call, solvers in flight)
export TMPDIR=/tmp
for cfg in "128 2" "128 3" "128 4" "192 3" "256 2" "96 4" "128 6"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline --lba-windows $1 --lba-inflight $2 --lba-calls 6 > gpurun_out/lbasw_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/lbasw_$1_$2.json'))['lba']; print('$1 x $2', d['value'], d['roofline']['frac'], d['host_plan_ms_per_call'])"
done
