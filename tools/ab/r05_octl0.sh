#!/bin/bash
# (1) LBA / shim / mapping GPU tests after the wave-uniform index changes; (2) k_octree's level-0
# launch with one wave per (frame, level) (default) vs SLAMHOT_OCT_L0=1 (4 waves, in-tree) vs
# SLAMHOT_OCT_L0=1 with 2 waves (lib/ab/libslamhot_oct2.so), interleaved headline / extract legs.
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py tests/test_gpu_mapping.py -x -q --timeout 120 --timeout-method thread > gpurun_out/octl0_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/octl0_tests.log; [ $rc -ne 0 ] && exit $rc
A=orb-slam3-noted_amd/lib/libslamhot.so; C=orb-slam3-noted_amd/lib/ab/libslamhot_oct2.so
for i in 1 2 3; do
  for cfg in "$A 0" "$A 1" "$C 1"; do
    set -- $cfg
    SLAMHOT_LIB=$1 SLAMHOT_OCT_L0=$2 timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/octl0.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/octl0.json'))
print('$1'.split('/')[-1], 'L0=$2', 'headline', d['value'], 'extract', d['extract']['value'], 'stages', d.get('headline_detail',{}).get('extractor_stage_ms_per_launch'))"
  done
done
