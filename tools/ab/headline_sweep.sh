#!/bin/bash
# headline batch-size / batches-in-flight sweep (bench.py --legs headline)
set -e
for cfg in "128 3" "256 2" "256 3" "192 3" "128 4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --legs headline --no-cpu-baseline --pairs $1 --inflight $2 > gpurun_out/hl_$1_$2.json 2>/dev/null
done
