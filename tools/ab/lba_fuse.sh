#!/bin/bash
# LBA small-batch fusion (point prep in k_iter_begin, trial error in k_trial_control): parity tests
# with the fused path forced on and off, then the drop-in latency and the single-window trace
export TMPDIR=/tmp
(cd tools/microbench && timeout -k 10 60 ./mb_ldlt) || exit 1
for F in 1 0; do
  SLAMHOT_LBA_FUSE=$F timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fuse_tests_$F.log 2>&1
  rc=$?; echo "fuse=$F tests rc=$rc: $(tail -1 gpurun_out/fuse_tests_$F.log)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 100 python tools/lba_dropin.py 16 --write-map /tmp/lba_map.bin || exit 1
SLAMHOT_LBA_FUSE=0 timeout -k 10 100 python tools/lba_dropin.py 16 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fuse_prof -o lba -- tests/cpp/shim_driver lbatime /tmp/lba_map.bin /tmp/lba_out.bin 4 > gpurun_out/fuse_prof.log 2>&1 || exit 1
f=$(find gpurun_out/fuse_prof -name "*kernel_trace.csv" | head -1); python3 tools/lba_calls.py $f | tail -2
