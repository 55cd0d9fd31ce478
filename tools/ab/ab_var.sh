#!/bin/bash
# A/B of experiment libraries with per-library parity: TESTS run against every library
# (SLAMHOT_LIB), then LEGS interleaved twice.  Usage: tools/ab/ab_var.sh TAG "TESTS" LEGS LIB...
export TMPDIR=/tmp
TAG=$1; TESTS=$2; LEGS=$3; shift 3
for L in "$@"; do
  SLAMHOT_LIB=$L timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/abv_tests_${TAG}_$(basename $L .so).log 2>&1
  rc=$?; echo "$(basename $L) tests_exit=$rc $(tail -1 gpurun_out/abv_tests_${TAG}_$(basename $L .so).log)"
  [ $rc -ne 0 ] && exit $rc
done
for i in 1 2 3; do
  for L in "$@"; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs $LEGS --no-cpu-baseline > gpurun_out/abv_$TAG.json 2>/dev/null || exit 1
    python3 - "$L" <<PY
import json, sys
d = json.load(open("gpurun_out/abv_$TAG.json"))
out = {"lib": sys.argv[1].split("/")[-1]}
if "value" in d:
    out["headline"] = d["value"]; hd = d.get("headline_detail", {})
    out["ext_stages"] = hd.get("extractor_stage_ms_per_launch")
    out["stages"] = hd.get("stage_ms_per_step")
for k in ("extract", "lba", "track", "projection", "localmap", "pose"):
    if k in d: out[k] = d[k]["value"]
if "extract" in d: out["extract_stages"] = d["extract"].get("stages_ms_per_step")
print(json.dumps(out))
PY
  done
done
