#!/bin/bash
# Extraction throughput vs batches in flight (and batch size) on one box.
export TMPDIR=/tmp
for cfg in "1 256" "2 256" "3 256" "4 256" "2 512" "3 128" "6 128"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --no-cpu-baseline --match-pairs 0 --lba-windows 0 --pose-frames 0 --stereo-pairs 0 \
    --inflight $1 --batch $2 > gpurun_out/if.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/if.json')); print('inflight=$1 batch=$2', d['value'], d['ms_per_step'])"
done
