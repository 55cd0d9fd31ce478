#!/bin/bash
# k_schur_rows and the other LBA kernels in isolation (one solver, one call) per library, then the
# LBA leg interleaved N times.  Usage: tools/ab/lba_iso_libs.sh N LIB...
export TMPDIR=/tmp
N=$1; shift
for L in "$@"; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iso/$n -o run -- python3 bench.py --legs lba --no-cpu-baseline --lba-inflight 1 --lba-calls 2 > gpurun_out/iso_$n.json 2>/dev/null || exit 1
  f=$(find gpurun_out/prof_iso/$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:5]: print(r['Name'][:40].ljust(40), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
done
for i in $(seq $N); do
  for L in "$@"; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline > gpurun_out/lbai.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lbai.json'))['lba']; print('$(basename $L)', d['value'], d['single_window']['ms_per_lm_iteration'])"
  done
done
