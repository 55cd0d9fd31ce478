#!/bin/bash
# Price each extractor stage inside the concurrent (3 batches in flight) pipeline: the bench
# value with that stage left out (experiment build, SLAMHOT_SKIP bitmask; results invalid).
# Stages: 0 resize, 1 fast, 2 octree, 3 layout, 4 orb.  Usage: tools/ab/stage_price.sh LIB
export TMPDIR=/tmp
LIB=${1:-tools/libslamhot_exp.so}
for m in 0 1 2 4 16 22 21 19; do
  SLAMHOT_LIB=$LIB SLAMHOT_SKIP=$m timeout -k 10 120 python bench.py --no-cpu-baseline --match-pairs 0 --lba-windows 0 \
    --pose-frames 0 --stereo-pairs 0 > gpurun_out/price_$m.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/price_$m.json')); print('skip=$m', d['value'], d['ms_per_step'])"
done
