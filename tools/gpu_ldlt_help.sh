#!/bin/bash
# helper-assisted LDL^T (k_ldlt_t16x): look-ahead / helper-count variants in the microbenchmark vs
# the one-workgroup kernel (x compared bit for bit), the LBA / shim parity tests, then the LBA leg
# (drop-in call) with and without the helpers
export TMPDIR=/tmp
TAG=${1:-h}
mkdir -p gpurun_out
OUT=gpurun_out/ldlt_help_$TAG.txt
cd tools/microbench
for v in la2 la3 la4 la6 la4 la3; do echo "== $v"; timeout -k 5 60 ./mb_ldlt_$v 288 30 | grep -v "ldlt " || exit 1; done 2>&1 | tee ../../$OUT
for n in 192 100 33 16; do timeout -k 5 60 ./mb_ldlt $n 20 | grep -v "ldlt " || exit 1; done 2>&1 | tee -a ../../$OUT
cd ../..
timeout -k 10 400 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  SLAMHOT_LDLT_HELP=$v timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline > gpurun_out/lba_help${v}_$TAG.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/lba_help${v}_$TAG.json'))['lba']; print('help=$v', 'lba', d['value'], 'drop_in', d['single_window']['drop_in']['wall_ms_per_call'], 'device', d['single_window']['drop_in']['device_ms'])" | tee -a $OUT
done
