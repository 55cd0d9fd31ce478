#!/bin/bash
# A/B of the XCD-aware workgroup order in k_fast_wave / k_orb3: extractor parity tests with the
# in-tree build, interleaved headline + extract legs of both libraries, then one FETCH_SIZE pass
# per library (headline leg, one batch in flight).  Args: tag.
export TMPDIR=/tmp
TAG=${1:-xcd}
A=orb-slam3-noted_amd/lib/ab/libslamhot_noxcd.so
B=orb-slam3-noted_amd/lib/libslamhot.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_stereo.py tests/test_gpu_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/ab_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 200 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/ab_$TAG.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_$TAG.json')); e=d['extract']
print(sys.argv[1].split('/')[-1], 'headline', d['value'], 'fast', d['roofline']['avg_launch_ms'], d['headline_detail']['extractor_stage_ms_per_launch'], 'extract', e['value'], e['stages_ms_per_step'])" $L
  done
done
for L in $A $B; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_$TAG/$n/p1 -o run -- python3 bench.py --legs headline --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$n.log 2>&1 || exit 1
  echo "== $n"; python3 tools/parse_counters.py gpurun_out/pmc_$TAG/$n | grep -E "k_fast_wave|k_orb3|k_resize|k_octree"
done
