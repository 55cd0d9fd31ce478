#!/bin/bash
# A/B the extraction bench line between experiment libraries in one box session, interleaved.
# Usage: tools/ab/ab.sh LIB_A LIB_B [rounds]
export TMPDIR=/tmp
A=$1; B=$2; R=${3:-3}
for i in $(seq $R); do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --match-pairs 0 --lba-windows 0 --pose-frames 0 \
      --stereo-pairs 0 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], d['value'], d['stages_ms_per_step'])" $L
  done
done
