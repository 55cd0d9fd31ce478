#!/bin/bash
# LBA leg: in-tree library vs lib/ab/libslamhot_head.so (tools/build_head.sh lba), interleaved
# (3 pairs), after the LBA / shim GPU tests on the in-tree library.
export TMPDIR=/tmp
TAG=${1:-lbahead}
A=orb-slam3-noted_amd/lib/libslamhot.so; B=${HEADLIB:-orb-slam3-noted_amd/lib/ab/libslamhot_head.so}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline > gpurun_out/$TAG.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/$TAG.json')); l=d['lba']
print('$L'.split('/')[-1], 'lba', l['value'], 'plan ms/call', l['host_plan_ms_per_call'], 'ms/call', l['ms_per_call'], 'dev 1 solver', l['device_lm_iters_per_s_one_solver'], 'drop-in', l['single_window']['drop_in']['wall_ms_per_call'])"
  done
done
