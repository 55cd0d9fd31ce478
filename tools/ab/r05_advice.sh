#!/bin/bash
# round 5: the advisor's test additions (threaded batch staging with a > 4096-feature frame, LBA stop at
# the optimize(5) boundary with 12 windows) and the shim / projection / LBA suites they touch
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_projection.py tests/test_gpu_lba.py tests/test_gpu_shim.py tests/test_gpu_cpp_host.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/advice_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" gpurun_out/advice_tests.log | tail -15; tail -3 gpurun_out/advice_tests.log; exit $rc
