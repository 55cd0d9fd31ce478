#!/bin/bash
# k_fast_wave with host-computed wave-cell records (FastWaveCell: scalar geometry, buffer-load
# staging with SGPR row offsets, no per-wave divisions) vs the previous commit's extractor
# (lib/ab/libslamhot_head.so): bit-exact tests, interleaved legs, issue counters + kernel times.
export TMPDIR=/tmp
A=orb-slam3-noted_amd/lib/libslamhot.so; B=orb-slam3-noted_amd/lib/ab/libslamhot_head.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py tests/test_gpu_stereo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fastvalu_tests.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/fastvalu_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for L in $A $B; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs headline,extract --no-cpu-baseline > gpurun_out/fastvalu.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/fastvalu.json'))
print('$L'.split('/')[-1], 'headline', d['value'], 'extract', d['extract']['value'], 'stage ms/launch', d.get('headline_detail',{}).get('extractor_stage_ms_per_launch'))"
  done
done
for L in $A $B; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d gpurun_out/fastvalu_pmc/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/fastvalu_pmc/$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections, os
for kern in ("k_fast_wave", "k_orb3"):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(sys.argv[1])):
        if kern in r["Kernel_Name"]: acc[r["Counter_Name"]] += float(r["Counter_Value"])
    st = [r for r in csv.DictReader(open(os.path.join(os.path.dirname(sys.argv[1]), "run_kernel_stats.csv"))) if kern in r["Name"]]
    w = max(1.0, acc["SQ_WAVES"])
    print(sys.argv[2], kern, "waves", round(w), "per wave: valu", round(acc["SQ_INSTS_VALU"] / w, 1), "salu", round(acc["SQ_INSTS_SALU"] / w, 1),
          "lds", round(acc["SQ_INSTS_LDS"] / w, 1), "wave_cycles", round(4 * acc["SQ_WAVE_CYCLES"] / w), "avg us", round(float(st[0]["AverageNs"]) / 1e3, 1) if st else None)
PY
done
SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_ftrace.so timeout -k 10 200 python bench.py --legs headline --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/ftrace.json 2> gpurun_out/ftrace.err || exit 1
grep -c "^FAST lvl" gpurun_out/ftrace.json
