#!/bin/bash
# PoseOptimization leg timed on pre-marshalled frames: pose parity tests, then the leg twice
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pose.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pose_tests.log 2>&1
rc=$?; echo "pose tests rc=$rc: $(tail -1 gpurun_out/pose_tests.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --legs pose --no-cpu-baseline > gpurun_out/pose.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/pose.json'))['pose']; print('pose', d['value'], d['ms_per_call'])"
done
