#!/bin/bash
# headline leg: extractor sub-streams (SLAMHOT_SUBSTREAMS) x batches in flight, interleaved twice
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "1 4" "2 4" "2 3" "4 2"; do
    set -- $cfg
    SLAMHOT_SUBSTREAMS=$1 timeout -k 10 200 python bench.py --legs headline,extract --no-cpu-baseline --inflight $2 > gpurun_out/ss.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ss.json')); print('substreams $1 inflight $2', d['value'], 'extract', d['extract']['value'])"
  done
done
