#!/bin/bash
# k_ldlt_t16: late panels keep wave 0's SIMD free of trailing-update waves (T16_SPARE_TILES = the
# trailing-tile count at or below which they sit out; 0 = never, the old kernel; 1000 = always):
# mb_ldlt per threshold, LBA parity on the default (48), isolated kernel stats and the drop-in call
export TMPDIR=/tmp
for r in 1 2; do for v in 0 48 96 1000; do
  echo -n "spare $v "; (cd tools/microbench && timeout -k 10 60 ./mb_ldlt_sp$v | grep t16) || exit 1
done; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/spare_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/spare_tests.log)"; [ $rc -ne 0 ] && exit $rc
L=orb-slam3-noted_amd/lib
bash tools/ab/lba_iso_libs.sh 1 $L/ab/libslamhot_sp0.so $L/libslamhot.so $L/ab/libslamhot_sp96.so $L/ab/libslamhot_sp1000.so || exit 1
timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | tail -4
