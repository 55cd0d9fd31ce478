#!/bin/bash
# LBA leg A/B over several library builds (args: tag lib1 lib2 ...), interleaved twice; parity
# tests with the in-tree build first.
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lba_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/lba_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for L in "$@"; do
    SLAMHOT_LIB=$L timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline > gpurun_out/lba_ab_$TAG.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/lba_ab_$TAG.json'))['lba']; print(sys.argv[1].split('/')[-1], d['value'], d['roofline']['frac'], d['device_lm_iters_per_s_one_solver'], d['host_plan_ms_per_call'], d['single_window'])" $L
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lba_tl_$TAG -o t -- python3 bench.py --legs lba --no-cpu-baseline > gpurun_out/lba_tl_$TAG.json 2>gpurun_out/lba_tl_$TAG.err || exit 1
python3 tools/busy.py gpurun_out/lba_tl_$TAG
