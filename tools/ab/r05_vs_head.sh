#!/bin/bash
# In-tree library vs lib/ab/libslamhot_head.so (tools/build_head.sh: the last commit's source of
# one file): the given GPU tests, interleaved headline / extract legs (3 pairs), and one rocprofv3
# kernel-stats pass per library (headline, one batch in flight).  Usage: r05_vs_head.sh TAG "TESTS"
export TMPDIR=/tmp
TAG=$1; TESTS=$2
A=orb-slam3-noted_amd/lib/libslamhot.so; B=${HEADLIB:-orb-slam3-noted_amd/lib/ab/libslamhot_head.so}
timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/$TAG.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/$TAG.json'))
print('$L'.split('/')[-1], 'headline', d['value'], 'extract', d['extract']['value'], 'stage ms/launch', d.get('headline_detail',{}).get('extractor_stage_ms_per_launch'))"
  done
done
for L in $A $B; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/${TAG}_prof/$n/run_kernel_stats.csv $n <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], [(r["Name"][:24], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1)) for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]])
PY
done
