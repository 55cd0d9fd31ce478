#!/bin/bash
# k_orb3 with fewer VALU instructions (in-tree) vs lib/ab/libslamhot_orbhead.so (the extractor of
# commit 460e84b): extractor bit-exact tests + smoke, interleaved headline / extract legs, k_orb3
# issue counters + kernel times per library, per-phase cycles of both trace builds.
export TMPDIR=/tmp
A=orb-slam3-noted_amd/lib/libslamhot.so; B=orb-slam3-noted_amd/lib/ab/libslamhot_orbhead.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orbvalu_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/orbvalu_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/orbvalu.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/orbvalu.json'))
print('$L'.split('/')[-1], 'headline', d['value'], 'extract', d['extract']['value'], 'stages', d.get('headline_detail',{}).get('stage_ms_per_step'))"
  done
done
for L in $A $B; do
  n=$(basename $L .so)
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT"; do
    SLAMHOT_LIB=$L timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv --pmc $grp -d gpurun_out/orbvalu_pmc/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
  done
  f=$(find gpurun_out/orbvalu_pmc/$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections, os
acc = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_orb3" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
st = [r for r in csv.DictReader(open(os.path.join(os.path.dirname(sys.argv[1]), "run_kernel_stats.csv"))) if "k_orb3" in r["Name"]]
w = max(1.0, acc["SQ_WAVES"])
print(sys.argv[2], {k: round(v) for k, v in acc.items()}, "per wave: valu", round(acc["SQ_INSTS_VALU"] / w, 1),
      "salu", round(acc["SQ_INSTS_SALU"] / w, 1), "lds", round(acc["SQ_INSTS_LDS"] / w, 1),
      "wave_cycles", round(4 * acc["SQ_WAVE_CYCLES"] / w), "k_orb3 avg us", round(float(st[0]["AverageNs"]) / 1e3, 1) if st else None)
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
