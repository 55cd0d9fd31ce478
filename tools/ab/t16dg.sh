#!/bin/bash
# k_ldlt_t16 with the diagonal tiles resident in LDS (in-tree) vs HEAD~ (lib/ab/libslamhot_base.so,
# tools/microbench/mb_ldlt_base): phase-timed factorization at n = 288, LBA parity, isolated kernel
# stats and the LBA leg interleaved, then the drop-in call
export TMPDIR=/tmp
cd tools/microbench
for r in 1 2; do
  echo -n "base "; timeout -k 10 60 ./mb_ldlt_base | grep t16 || exit 1
  echo -n "dg   "; timeout -k 10 60 ./mb_ldlt | grep t16 || exit 1
done
cd ../..
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t16dg_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t16dg_tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab/lba_iso_libs.sh 2 orb-slam3-noted_amd/lib/ab/libslamhot_base.so orb-slam3-noted_amd/lib/libslamhot.so || exit 1
timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | tail -4
