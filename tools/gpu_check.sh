#!/bin/bash
# Round-end style check: all GPU parity tests, smoke(), then the driver's exact bench command
# (python3 bench.py --gpus 1 --steps 20 --warmup 5), each step under its own time limit.
export TMPDIR=/tmp
TAG=${1:-c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
cat gpurun_out/smoke_$TAG.log
bash tools/gpu_bench_driver.sh "$TAG"
