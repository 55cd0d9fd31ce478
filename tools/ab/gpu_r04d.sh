#!/bin/bash
# round 4 evidence: LBA / shim parity first (device-side optimize(5) -> optimize(10) transition),
# then the round profile (kernel stats, one batch in flight, PMC, LBA FP64) and the drop-in trace
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py tests/test_gpu_cpp_host.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_lba_tests.log 2>&1
rc=$?; echo "lba tests rc=$rc: $(tail -1 gpurun_out/r04d_lba_tests.log)"; [ $rc -ne 0 ] && exit $rc
SLAMHOT_LBA_TRACE=1 timeout -k 10 100 python tools/lba_dropin.py 16 2>&1 | tail -8 || exit 1
SKIP_CAL=1 bash tools/profile_round.sh r04d || exit 1
bash tools/lba_dropin_prof.sh gpurun_out/dropin_r04d || exit 1
echo r04d_done
