#!/bin/bash
# LBA A/B on the GPU box: parity tests with the tile LDL^T, then the throughput probe for the
# tile kernel and the panel kernel (SLAMHOT_LDLT=panel), then a kernel trace of one batch of 1 and 64.
export TMPDIR=/tmp
TAG=${1:-ab}
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_cpp_host.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lba_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/lba_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/lba_bench.py --batches 1,8,64,128 > gpurun_out/lba_bench_${TAG}_t16.log 2>&1 || exit 1
SLAMHOT_LDLT=panel timeout -k 10 200 python tools/lba_bench.py --batches 1,8,64,128 > gpurun_out/lba_bench_${TAG}_panel.log 2>&1 || exit 1
for f in t16 panel; do echo "== $f"; cat gpurun_out/lba_bench_${TAG}_$f.log; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lba_prof_$TAG -o lba -- python3 tools/lba_bench.py --batches 1,64 --reps 1 > gpurun_out/lba_prof_$TAG.log 2>&1 || exit 1
python3 tools/kernel_split.py gpurun_out/lba_prof_$TAG 2>/dev/null | head -40
