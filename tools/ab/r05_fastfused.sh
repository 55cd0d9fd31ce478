#!/bin/bash
# k_fast_wave with passes A / B1 / B run once at min(iniThFAST, minThFAST) and pass C applying
# both thresholds (in-tree) vs the two-attempt form (lib/ab/libslamhot_nofused.so): extractor,
# frame and stereo bit-exact tests, interleaved headline / extract legs, kernel stats per library,
# per-pass cycles of both trace builds.
export TMPDIR=/tmp
A=orb-slam3-noted_amd/lib/libslamhot.so; B=orb-slam3-noted_amd/lib/ab/libslamhot_nofused.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py tests/test_gpu_stereo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fastfused_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/fastfused_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/fastfused.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/fastfused.json'))
print('$L'.split('/')[-1], 'headline', d['value'], 'extract', d['extract']['value'], 'fast ms/launch', d.get('headline_detail',{}).get('extractor_stage_ms_per_launch'))"
  done
done
for L in $A $B; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fastfused_prof/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/fastfused_prof/$n/run_kernel_stats.csv $n <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], [(r["Name"][:22], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1)) for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:6]])
PY
done
for T in ftrace ftrace0; do
  SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_$T.so timeout -k 10 200 python bench.py --legs headline --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/$T.json 2> gpurun_out/$T.err || exit 1
  grep "^FAST lvl" gpurun_out/$T.json > gpurun_out/$T.txt
  python3 - gpurun_out/$T.txt $T <<'PY'
import re, collections, sys
rows = []
for l in open(sys.argv[1]):
    d = {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", l)}
    d.update({k: int(v) for k, v in re.findall(r" (zero|A|B1|B|C) (\d+)", l)})
    rows.append(d)
tot = collections.Counter()
for r in rows:
    for f in ("zero", "A", "B1", "B", "C"): tot[f] += r[f]
n = max(1, len(rows))
print(sys.argv[2], "cells", len(rows), {f: round(tot[f] / n) for f in tot}, "total/cell", round(sum(tot.values()) / n))
PY
done
