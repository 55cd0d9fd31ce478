#!/bin/bash
# GPU iteration helper: parity tests, then serial (isolated stages) and concurrent bench.
export TMPDIR=/tmp
TAG=${1:-q}
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
SLAMHOT_SERIAL=1 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_s.json 2>gpurun_out/bench_${TAG}_s.err || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2>gpurun_out/bench_$TAG.err || exit 1
python3 - <<PY
import json
for f in ["gpurun_out/bench_${TAG}_s.json","gpurun_out/bench_${TAG}.json"]:
    d=json.load(open(f)); print(d["value"], {k: round(v,3) for k,v in d["stages_ms_per_step"].items()})
PY
