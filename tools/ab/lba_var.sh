#!/bin/bash
# isolated LBA kernel times (rocprofv3 kernel trace, one solver in flight) for each library
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lv/$n -o run -- python3 bench.py --legs lba --no-cpu-baseline --lba-inflight 1 --lba-calls 1 --steps 3 --warmup 1 > gpurun_out/lv_$n.json 2>/dev/null || exit 1
  f=$(find gpurun_out/prof_lv/$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:5]: print(r['Name'][:40].ljust(40), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
done
