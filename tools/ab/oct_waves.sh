#!/bin/bash
# single-frame extraction latency per octree wave count (variant libraries) + their parity tests
export TMPDIR=/tmp
for L in orb-slam3-noted_amd/lib/libslamhot.so orb-slam3-noted_amd/lib/ab/libslamhot_ow8.so orb-slam3-noted_amd/lib/ab/libslamhot_ow16.so; do
  SLAMHOT_LIB=$L timeout -k 10 200 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ow_tests_$(basename $L .so).log 2>&1 || { echo "$L tests failed"; exit 1; }
  for i in 1 2; do SLAMHOT_LIB=$L timeout -k 10 120 python3 tools/single_frame.py | sed "s|^|$(basename $L) |" || exit 1; done
done
