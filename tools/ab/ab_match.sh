#!/bin/bash
# A/B the match leg (extract + ComputeBoW + SearchByBoW) between two builds on one box.
export TMPDIR=/tmp
for i in 1 2; do for L in $1 $2; do
SLAMHOT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --lba-windows 0 --pose-frames 0 --stereo-pairs 0 > gpurun_out/abm.json 2>/dev/null || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/abm.json')); print(sys.argv[1], d['value'], d['match']['value'], d['match']['ms_per_step'])" $L
done; done
