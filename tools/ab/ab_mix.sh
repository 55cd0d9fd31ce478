#!/bin/bash
# A/B of (library, environment) pairs: TESTS once per entry, then LEGS interleaved three times.
# Entry = LIB or LIB@VAR=value.  Usage: tools/ab/ab_mix.sh TAG "TESTS" LEGS ENTRY...
export TMPDIR=/tmp
TAG=$1; TESTS=$2; LEGS=$3; shift 3
run() {  # entry, command...
  local E=$1; shift
  local L=${E%%@*} V=""
  [ "$E" != "$L" ] && V=${E#*@}
  env SLAMHOT_LIB=$L $V "$@"
}
for E in "$@"; do
  n=$(echo "$E" | tr '=/@ ' '____')
  run "$E" timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/abm_tests_${TAG}_$n.log 2>&1
  rc=$?; echo "$E tests_exit=$rc $(tail -1 gpurun_out/abm_tests_${TAG}_$n.log)"
  [ $rc -ne 0 ] && exit $rc
done
for i in 1 2 3; do
  for E in "$@"; do
    run "$E" timeout -k 10 300 python bench.py --legs $LEGS --no-cpu-baseline > gpurun_out/abm_$TAG.json 2>/dev/null || exit 1
    python3 - "$E" <<PY
import json, sys
d = json.load(open("gpurun_out/abm_$TAG.json"))
out = {"entry": sys.argv[1].split("/")[-1]}
if "value" in d:
    out["headline"] = d["value"]; hd = d.get("headline_detail", {})
    out["stages"] = hd.get("stage_ms_per_step")
for k in ("extract", "lba", "track", "projection", "localmap", "pose"):
    if k in d: out[k] = d[k]["value"]
print(json.dumps(out))
PY
  done
done
