#!/bin/bash
# t16_diag two-row form (SLAMHOT_T16_DIAG2=1: A and I halves in DPP rows 0 / 1, multiplier local,
# one v_permlane16_swap for the I half; =2: the same with the chain scheduled ahead by hand) vs
# the four-group form: per-tile microbench with output hashes, the whole factorization at
# n = 288, LBA parity per variant library, LBA leg interleaved
export TMPDIR=/tmp
cd tools/microbench
for r in 1 2; do
  for v in "" 2 3; do
    echo "== diag$v"; timeout -k 10 60 ./mb_diag$v || exit 1; timeout -k 10 60 ./mb_ldlt$v | grep t16 || exit 1
  done
done
cd ../..
for v in diag2 diag3; do
  SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${v}_tests.log 2>&1
  rc=$?; echo "$v tests rc=$rc: $(tail -1 gpurun_out/${v}_tests.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/ab/lba_iso_libs.sh 2 orb-slam3-noted_amd/lib/libslamhot.so orb-slam3-noted_amd/lib/ab/libslamhot_diag2.so orb-slam3-noted_amd/lib/ab/libslamhot_diag3.so || exit 1
