#!/bin/bash
# round 4f: LBA / shim / C++ host parity with the packed step tally and the control blocks loaded ahead, then the
# drop-in latency, its phase trace and its kernel trace
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py tests/test_gpu_cpp_host.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_lba_tests.log 2>&1
rc=$?; echo "lba tests rc=$rc: $(tail -1 gpurun_out/r04f_lba_tests.log)"; [ $rc -ne 0 ] && exit $rc
SLAMHOT_LBA_TRACE=1 timeout -k 10 100 python tools/lba_dropin.py 6 2>&1 | tail -12 || exit 1
timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | tail -5 || exit 1
bash tools/lba_dropin_prof.sh gpurun_out/dropin_r04f || exit 1
echo r04f_done
