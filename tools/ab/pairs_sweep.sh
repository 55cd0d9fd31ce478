#!/bin/bash
# headline leg: pairs per step x batches in flight, interleaved twice
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "128 4" "192 4" "256 3" "256 4" "192 3"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --legs headline --no-cpu-baseline --pairs $1 --inflight $2 > gpurun_out/ps.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ps.json')); print('pairs $1 inflight $2', d['value'], d['ms_per_step'])"
  done
done
