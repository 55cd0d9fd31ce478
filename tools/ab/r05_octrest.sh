#!/bin/bash
# k_octree multi-wave (4 waves per (frame, level)) for the level-0 group (SLAMHOT_OCT_L0) and the
# levels 1-7 group (SLAMHOT_OCT_REST) of the batch pipeline: tests with both on, then the four
# settings interleaved on the headline / extract legs.
export TMPDIR=/tmp
SLAMHOT_OCT_L0=1 SLAMHOT_OCT_REST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > gpurun_out/octrest_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/octrest_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    SLAMHOT_OCT_L0=$1 SLAMHOT_OCT_REST=$2 timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/octrest.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/octrest.json'))
print('L0=$1 REST=$2', 'headline', d['value'], 'extract', d['extract']['value'], 'octree', d.get('headline_detail',{}).get('extractor_stage_ms_per_launch',{}).get('k_octree'))"
  done
done
