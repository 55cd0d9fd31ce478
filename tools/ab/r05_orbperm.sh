#!/bin/bash
# k_orb3 A/B: the in-tree build vs lib/ab/libslamhot_orbhead.so (the previous commit's extractor)
# and lib/ab/libslamhot_orbperm2.so (SLAMHOT_ORB_PERM=2, the per-angle-bin bit order): extractor
# bit-exact tests, interleaved headline / extract legs, k_orb3 LDS counters + kernel times per
# library, per-phase cycles of the trace builds (libslamhot_orbtrace / _orbheadtr).
export TMPDIR=/tmp
A=orb-slam3-noted_amd/lib/libslamhot.so; B=orb-slam3-noted_amd/lib/ab/libslamhot_orbhead.so; C=orb-slam3-noted_amd/lib/ab/libslamhot_orbperm2.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orbperm_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -2 gpurun_out/orbperm_tests.log; [ $rc -ne 0 ] && exit $rc
SLAMHOT_LIB=$C timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orbperm2_tests.log 2>&1
rc=$?; echo perm2_tests_exit=$rc; tail -2 gpurun_out/orbperm2_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for L in $A $B $C; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/orbperm.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/orbperm.json'))
print('$L'.split('/')[-1], 'headline', d['value'], 'extract', d['extract']['value'], 'stages', d.get('headline_detail',{}).get('stage_ms_per_step'))"
  done
done
for L in $A $B $C; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES -d gpurun_out/orbperm_pmc/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/orbperm_pmc/$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections, os
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_orb3" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
st = [r for r in csv.DictReader(open(os.path.join(os.path.dirname(sys.argv[1]), "run_kernel_stats.csv"))) if "k_orb3" in r["Name"]]
print(sys.argv[2], {k: round(v) for k, v in acc.items()}, "conflict/active", round(acc["SQ_LDS_BANK_CONFLICT"] / max(1, acc["SQ_ACTIVE_INST_LDS"]), 3),
      "k_orb3 avg us", round(float(st[0]["AverageNs"]) / 1e3, 1) if st else None)
PY
done
for T in orbtrace orbheadtr; do
  SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_$T.so timeout -k 10 200 python bench.py --legs headline --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/$T.json 2> gpurun_out/$T.err || exit 1
  grep "ORB slot" gpurun_out/$T.json | head -400 > gpurun_out/$T.txt
  python3 - gpurun_out/$T.txt $T <<'PY'
import re, collections, sys
tot = collections.defaultdict(list)
names = ("pro", "stage", "ic", "horiz", "sincos", "desc")
for l in open(sys.argv[1]):
    m = re.search(r"l=(\d+)(?: pro (\d+))? stage (\d+) ic (\d+) horiz (\d+) sincos (\d+) desc (\d+)", l)
    if m:
        for k, v in zip(names, m.groups()[1:]):
            if v is not None: tot[k].append(int(v))
print(sys.argv[2], {k: (len(v), sorted(v)[len(v) // 2], round(sum(v) / len(v))) for k, v in tot.items()})
PY
done
