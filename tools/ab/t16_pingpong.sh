#!/bin/bash
# k_ldlt_t16 trailing loop with ping-pong tile registers (no `cur = nxt` copy that waited for the
# prefetch) vs HEAD (lib/ab/libslamhot_base.so, tools/microbench/mb_ldlt_base): mb_ldlt at three
# sizes, LBA / shim parity, isolated kernel stats and the LBA leg per library, the drop-in call
export TMPDIR=/tmp
for n in 288 192 100; do for b in mb_ldlt_base mb_ldlt; do
  echo -n "$b "; (cd tools/microbench && timeout -k 10 60 ./$b $n | grep t16) || exit 1
done; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pingpong_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/pingpong_tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab/lba_iso_libs.sh 2 orb-slam3-noted_amd/lib/ab/libslamhot_base.so orb-slam3-noted_amd/lib/libslamhot.so || exit 1
timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | tail -4
