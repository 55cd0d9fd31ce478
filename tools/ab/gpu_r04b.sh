#!/bin/bash
# round 4: matcher host-buffer paths (device grid, pipelined staging), LBA drop-in overlap hook
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_projection.py tests/test_gpu_shim.py tests/test_gpu_pose.py tests/test_gpu_lba.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04b_tests.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python tools/lba_dropin.py 16 || exit 1
timeout -k 10 300 python bench.py --legs localmap,projection --no-cpu-baseline > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r04b_bench.json'))
for k in ('localmap','projection'):
    x=d[k]; print(k, x['value'], x['ms_per_call'], x.get('call_split'))
    if 'keyframe_variant' in x: print('  kf', x['keyframe_variant'])
"
