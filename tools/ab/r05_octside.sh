#!/bin/bash
# k_octree's level-0 group on a side stream beside levels 1-7 (SLAMHOT_OCT_SIDE=1, default) vs one
# after the other (=0): extractor tests, interleaved headline / extract legs.
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > gpurun_out/octside_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/octside_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    SLAMHOT_OCT_SIDE=$v timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/octside.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/octside.json'))
print('side=$v', 'headline', d['value'], 'extract', d['extract']['value'])"
  done
done
