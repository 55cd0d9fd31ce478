#!/bin/bash
# headline at 4 batches in flight: extractor A/B switches (multi-wave octree for level 0, chained FAST ranges)
export TMPDIR=/tmp
for r in 1 2; do
  for e in "X=0" "SLAMHOT_OCT_L0=1" "SLAMHOT_CHAIN_FAST=1"; do
    env $e timeout -k 10 200 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/he.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/he.json')); print('$e', d['value'], 'extract', d['extract']['value'])"
  done
done
