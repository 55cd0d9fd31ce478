#!/bin/bash
# A/B the LBA bench leg between two library builds (interleaved, one box session).
export TMPDIR=/tmp
A=$1; B=$2; R=${3:-2}
for i in $(seq $R); do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --match-pairs 0 --pose-frames 0 \
      --stereo-pairs 0 --lba-calls 6 > gpurun_out/ab_lba.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_lba.json'))['lba']; print(sys.argv[1], d['value'], d['device_lm_iters_per_s_one_solver'], d['single_window'])" $L
  done
done
