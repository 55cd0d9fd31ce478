#!/bin/bash
# A/B of runtime switches (environment assignments) on the in-tree build: TESTS once per
# setting, LEGS interleaved three times, then one rocprofv3 kernel-stats pass of PROF_LEGS per
# setting.  Usage: tools/ab/ab_env.sh TAG "TESTS" LEGS "VAR=a" "VAR=b" ...   ("-" = no assignment)
export TMPDIR=/tmp
TAG=$1; TESTS=$2; LEGS=$3; shift 3
PROF_LEGS=${PROF_LEGS:-$LEGS}
for E in "$@"; do
  n=$(echo "$E" | tr '=/ ' '___')
  env $( [ "$E" != "-" ] && echo "$E" ) timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/abe_tests_${TAG}_$n.log 2>&1
  rc=$?; echo "$E tests_exit=$rc $(tail -1 gpurun_out/abe_tests_${TAG}_$n.log)"
  [ $rc -ne 0 ] && exit $rc
done
for i in 1 2 3; do
  for E in "$@"; do
    env $( [ "$E" != "-" ] && echo "$E" ) timeout -k 10 300 python bench.py --legs $LEGS --no-cpu-baseline > gpurun_out/abe_$TAG.json 2>/dev/null || exit 1
    python3 - "$E" <<PY
import json, sys
d = json.load(open("gpurun_out/abe_$TAG.json"))
out = {"env": sys.argv[1]}
if "value" in d: out["headline"] = d["value"]
for k in ("extract", "lba", "track", "projection", "localmap", "pose"):
    if k in d: out[k] = d[k]["value"]
if "lba" in d: out["lba_single_ms_per_it"] = d["lba"]["single_window"]["ms_per_lm_iteration"]
print(json.dumps(out))
PY
  done
done
for E in "$@"; do
  n=$(echo "$E" | tr '=/ ' '___')
  if [ "$E" != "-" ]; then export "$E"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/$n -o run -- python3 bench.py --legs $PROF_LEGS --no-cpu-baseline --steps 5 --warmup 2 > /dev/null 2>&1 || exit 1
  if [ "$E" != "-" ]; then unset "${E%%=*}"; fi
  f=$(find gpurun_out/prof_$TAG/$n -name "*kernel_stats.csv" | head -1)
  echo "== $E"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]: print(r['Name'][:50].ljust(50), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
done
