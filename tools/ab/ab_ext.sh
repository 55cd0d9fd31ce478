#!/bin/bash
# Extractor A/B: GPU extractor / stereo / cpp tests with the in-tree build, then the headline and
# extract legs for each library (args: tag lib...), interleaved twice.
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_stereo.py tests/test_gpu_cpp_host.py tests/test_gpu_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ext_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/ext_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for L in "$@"; do
    SLAMHOT_LIB=$L timeout -k 10 200 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/ab_ext_$TAG.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_ext_$TAG.json')); e=d['extract']
print(sys.argv[1].split('/')[-1], 'headline', d['value'], 'fast', d['roofline']['avg_launch_ms'], d['headline_detail']['extractor_stage_ms_per_launch'], 'extract', e['value'], e['stages_ms_per_step'])" $L
  done
done
