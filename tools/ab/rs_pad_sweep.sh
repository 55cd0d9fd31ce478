#!/bin/bash
# FAST ROI row-stride probe: headline + extract legs at SLAMHOT_FAST_RS_PAD = 0..3 dwords,
# interleaved twice; the extractor bit-exact tests at pad 1 first.  Output: gpurun_out/rs_pad/
set -e
mkdir -p gpurun_out/rs_pad
SLAMHOT_FAST_RS_PAD=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_extractor.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/rs_pad/tests_pad1.log 2>&1
for rep in 1 2; do
  for pad in 0 1 2 3; do
    SLAMHOT_FAST_RS_PAD=$pad timeout -k 10 240 python3 bench.py --legs headline,extract --steps 50 --warmup 5 --no-cpu-baseline \
      > gpurun_out/rs_pad/pad${pad}_r${rep}.json 2> gpurun_out/rs_pad/pad${pad}_r${rep}.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/rs_pad/pad${pad}_r${rep}.json')); print('pad $pad rep $rep', round(d['value']), round(d['extract']['value']), d['roofline']['avg_launch_ms'])"
  done
done
