#!/bin/bash
# Headline + extract legs of several libraries, interleaved (3 rounds), then one rocprofv3 kernel-stats
# pass per library (headline, one batch in flight).  Usage: r05_libs.sh TAG LIB [LIB ...]
export TMPDIR=/tmp
TAG=$1; shift
for i in 1 2 3; do
  for L in "$@"; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/$TAG.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/$TAG.json'))
print('$L'.split('/')[-1], 'headline', d['value'], 'extract', d['extract']['value'], 'stages', d.get('headline_detail',{}).get('stage_ms_per_step'))"
  done
done
for L in "$@"; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/${TAG}_prof/$n/run_kernel_stats.csv $n <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], [(r["Name"][:28], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1)) for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9]])
PY
done
