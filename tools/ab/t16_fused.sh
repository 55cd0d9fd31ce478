#!/bin/bash
# k_ldlt_t16 round 5 (panel TRSM fused into the previous panel's trailing update, one barrier per
# panel, next diagonal tile via LDS, flag-driven back-solve) vs the round-4 kernel (mb_ldlt_prev,
# built from the previous commit's lba.hip): time per n and x bit for bit, then the LBA / shim
# parity tests and the drop-in call
export TMPDIR=/tmp
cd tools/microbench
timeout -k 5 60 ./mb_diag || exit 1
for n in 288 192 100 33 16; do
  timeout -k 5 60 ./mb_ldlt $n 20 /tmp/x_new_$n.bin | grep t16 || exit 1
  timeout -k 5 60 ./mb_ldlt_prev $n 20 /tmp/x_old_$n.bin | grep t16 || exit 1
  cmp /tmp/x_new_$n.bin /tmp/x_old_$n.bin && echo "n=$n x bit-identical"
done
for r in 1 2; do timeout -k 5 60 ./mb_ldlt 288 50 | grep t16; timeout -k 5 60 ./mb_ldlt_prev 288 50 | grep t16; done
cd ../..
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t16f_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t16f_tests.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | tail -4
timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline > gpurun_out/t16f_lba.json 2> gpurun_out/t16f_lba.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/t16f_lba.json'))['lba']; print('lba', d['value'], d['roofline']['frac'], d['single_window']['drop_in']['wall_ms_per_call'])"
