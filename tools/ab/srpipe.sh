#!/bin/bash
# k_schur_rows software-pipelined off-diagonal loop (SLAMHOT_SR_PIPE=1) vs base: LBA parity tests
# per library, isolated kernel stats, LBA leg interleaved; then the matcher legs (prepared calls)
export TMPDIR=/tmp
B=orb-slam3-noted_amd/lib/ab/libslamhot_base.so; V=orb-slam3-noted_amd/lib/ab/libslamhot_srpipe.so
SLAMHOT_LIB=$V SLAMHOT_SCHUR=rows timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py -x -q --timeout 120 --timeout-method thread > gpurun_out/srpipe_tests.log 2>&1
rc=$?; echo "srpipe tests rc=$rc: $(tail -1 gpurun_out/srpipe_tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab/lba_iso_libs.sh 2 $B $V || exit 1
timeout -k 10 300 python bench.py --legs localmap,projection --no-cpu-baseline > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r04c_bench.json'))
for k in ('localmap','projection'):
    x=d[k]; print(k, x['value'], x['ms_per_call'], x.get('call_split',{}).get('kernel_share'), x.get('call_split',{}).get('device_span_ms'))
    if 'keyframe_variant' in x: print('  kf', x['keyframe_variant']['value'], x['keyframe_variant']['ms_per_call'])
"
