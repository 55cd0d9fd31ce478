#!/bin/bash
# Host-code sanitizer pass (ASan + UBSan; GPU code is not instrumented): builds `make sanitize`,
# then runs the CPU test suite against the sanitized oracle (preloaded runtimes, leak checks off
# for the Python process) and the sanitized shim driver.  On a GPU box, `--gpu` also runs the
# C++ host-layer tests through the sanitized host_driver.
set -e
cd "$(dirname "$0")/.."
make -s sanitize
RT="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0
export SLAMHOT_ORACLE_LIB=oracle/build/liboracle_asan.so SLAMHOT_SHIM_DRIVER=tests/cpp/shim_driver_asan
LD_PRELOAD="$RT" python -m pytest tests -x -q -m "not gpu" -p no:xdist
if [ "$1" = "--gpu" ]; then
  SLAMHOT_HOST_DRIVER=tests/cpp/host_driver_asan LD_PRELOAD="$RT" \
    timeout -k 10 600 python -u -m pytest tests/test_gpu_cpp_host.py tests/test_gpu_shim.py -x -q --timeout 300 --timeout-method thread
fi
