export TMPDIR=/tmp
for n in 288 192 100; do (cd tools/microbench && timeout -k 10 60 ./mb_ldlt $n | grep -E "t16|reg") || exit 1; done
SLAMHOT_LDLT=reg timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ldlt_reg2_tests.log 2>&1
rc=$?; echo "reg tests rc=$rc: $(tail -1 gpurun_out/ldlt_reg2_tests.log)"; exit $rc
