#!/bin/bash
# Generic A/B of experiment libraries: GPU tests (TESTS, space-separated, in-tree build), then
# interleaved bench runs of each library (LEGS), then one rocprofv3 kernel-stats pass per library
# (headline leg, one batch in flight).  Usage: tools/ab/ab_libs.sh TAG "TESTS" LEGS LIB...
export TMPDIR=/tmp
TAG=$1; TESTS=$2; LEGS=$3; shift 3
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/ab_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for L in "$@"; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs $LEGS --no-cpu-baseline > gpurun_out/ab_$TAG.json 2>/dev/null || exit 1
    python3 - "$L" <<PY
import json, sys
d = json.load(open("gpurun_out/ab_$TAG.json"))
out = {"lib": sys.argv[1].split("/")[-1]}
if "value" in d: out["headline"] = d["value"]; out["stages"] = d.get("headline_detail", {}).get("stage_ms_per_step")
for k in ("extract", "lba", "track", "projection", "localmap", "pose"):
    if k in d: out[k] = d[k]["value"]
print(json.dumps(out))
PY
  done
done
for L in "$@"; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/prof_$TAG/$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]: print(r['Name'][:50].ljust(50), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
done
