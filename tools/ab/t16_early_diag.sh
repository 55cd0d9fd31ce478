#!/bin/bash
# k_ldlt_t16: wave 0 starts the next diagonal tile right after its own phase-(3) tile (the others
# wait for all sixteen phase-(3) arrivals on an LDS counter instead of a workgroup barrier) vs
# HEAD: mb_ldlt, LBA / shim parity, isolated kernel stats, the drop-in call
export TMPDIR=/tmp
for r in 1 2; do for n in 288 192; do for b in mb_ldlt_base mb_ldlt; do
  echo -n "$b "; (cd tools/microbench && timeout -k 10 60 ./$b $n | grep t16) || exit 1
done; done; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py tests/test_gpu_cpp_host.py -x -q --timeout 120 --timeout-method thread > gpurun_out/early_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/early_tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab/lba_iso_libs.sh 1 orb-slam3-noted_amd/lib/ab/libslamhot_base.so orb-slam3-noted_amd/lib/libslamhot.so || exit 1
timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | tail -4
