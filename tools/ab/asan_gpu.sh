#!/bin/bash
# Host-code ASan + UBSan over the library's C++ host side on the GPU box: lib/asan/libslamhot.so
# (hipcc, -Xarch_host -fsanitize=address,undefined, clang runtime) under the C++ host-layer and
# shim drivers built with clang++ -fsanitize=address,undefined -shared-libasan (the executable
# loads the runtime first; no preload).  GPU code is not instrumented.
export TMPDIR=/tmp
export ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
SLAMHOT_SHIM_DRIVER=tests/cpp/shim_driver_casan SLAMHOT_HOST_DRIVER=tests/cpp/host_driver_casan \
  timeout -k 10 900 python -u -m pytest tests/test_gpu_cpp_host.py tests/test_gpu_shim.py -x -q --timeout 300 --timeout-method thread > gpurun_out/asan_gpu.log 2>&1
rc=$?; echo "asan rc=$rc: $(tail -1 gpurun_out/asan_gpu.log)"; grep -m5 -E "ERROR: AddressSanitizer|runtime error" gpurun_out/asan_gpu.log; exit $rc
