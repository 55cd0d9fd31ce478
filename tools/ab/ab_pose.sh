#!/bin/bash
# A/B the PoseOptimization leg between two builds on one box.
export TMPDIR=/tmp
for i in 1 2; do for L in $1 $2; do
SLAMHOT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --match-pairs 0 --lba-windows 0 --stereo-pairs 0 > gpurun_out/abp.json 2>/dev/null || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/abp.json')); print(sys.argv[1], d['pose']['value'], d['pose']['ms_per_call'])" $L
done; done
