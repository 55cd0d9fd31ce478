#!/bin/bash
# headline and extract legs at 3 / 4 / 5 batches in flight, interleaved three times
export TMPDIR=/tmp
for r in 1 2 3; do
  for n in 3 4 5; do
    timeout -k 10 200 python bench.py --legs headline,extract --no-cpu-baseline --inflight $n > gpurun_out/if.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/if.json')); print('inflight $n headline', d['value'], 'extract', d['extract']['value'])"
  done
done
