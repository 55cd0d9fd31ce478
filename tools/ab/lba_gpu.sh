#!/bin/bash
# GPU iteration helper for the LBA path: parity tests, throughput probe, kernel trace summary.
export TMPDIR=/tmp
TAG=${1:-l}
timeout -k 10 400 python -m pytest tests/test_gpu_lba.py -x -q > gpurun_out/lba_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/lba_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/lba_bench.py ${LBA_BENCH_ARGS:---batches 1,8,64,128} > gpurun_out/lba_bench_$TAG.log 2>&1 || exit 1
cat gpurun_out/lba_bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lba_prof_$TAG -o lba -- python3 tools/lba_bench.py --batches 1,64 --reps 1 > gpurun_out/lba_prof_$TAG.log 2>&1 || exit 1
python3 tools/kernel_split.py gpurun_out/lba_prof_$TAG
