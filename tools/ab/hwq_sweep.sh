#!/bin/bash
# headline leg: hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) x batches in flight,
# interleaved twice
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "4 3" "8 3" "8 4" "8 6" "4 4"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python bench.py --legs headline --no-cpu-baseline --inflight $2 > gpurun_out/hwq.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/hwq.json')); print('hwq $1 inflight $2', d['value'], d['ms_per_step'])"
  done
done
