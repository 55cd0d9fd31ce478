#!/bin/bash
# Round-end style check: all GPU parity tests, smoke(), then the default bench line.
export TMPDIR=/tmp
TAG=${1:-c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
cat gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2>gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
