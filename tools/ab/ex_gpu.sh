#!/bin/bash
# GPU iteration helper for the extractor: parity tests, serial + concurrent bench (no LBA leg).
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 400 python -m pytest tests/test_gpu_extractor.py tests/test_golden.py -x -q > gpurun_out/ex_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/ex_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
SLAMHOT_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --lba-windows 0 > gpurun_out/exb_${TAG}_s.json 2>gpurun_out/exb_${TAG}_s.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --lba-windows 0 > gpurun_out/exb_$TAG.json 2>gpurun_out/exb_$TAG.err || exit 1
python3 - <<PY
import json
for f in ["gpurun_out/exb_${TAG}_s.json","gpurun_out/exb_${TAG}.json"]:
    d=json.load(open(f)); print(d["value"], {k: round(v,3) for k,v in d["stages_ms_per_step"].items()})
PY
