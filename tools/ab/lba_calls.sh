#!/bin/bash
# LBA leg: calls per solver in the timed region (6 vs 20: the solver start stagger and the tail
# are a smaller share of a longer window), interleaved three times
export TMPDIR=/tmp
for r in 1 2 3; do
  for c in 6 20; do
    timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline --lba-calls $c > gpurun_out/lc.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lc.json'))['lba']; print('calls $c', d['value'], d['ms_per_call'])"
  done
done
