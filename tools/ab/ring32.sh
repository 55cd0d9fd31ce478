#!/bin/bash
# FAST circle bytes as dwords (SLAMHOT_FAST_RING32) vs base: extractor parity per library, headline /
# extract legs interleaved, then one PMC pass per library over the headline (k_fast_wave LDS / VALU)
export TMPDIR=/tmp
B=orb-slam3-noted_amd/lib/ab/libslamhot_base.so; V=orb-slam3-noted_amd/lib/ab/libslamhot_ring32.so
bash tools/ab/ab_var.sh ring "tests/test_gpu_extractor.py tests/test_gpu_stereo.py" headline,extract $B $V || exit 1
for L in $B $V; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d gpurun_out/ring_pmc/$n -o run -- python3 bench.py --legs headline --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 > gpurun_out/ring_pmc_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/ring_pmc/$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_fast_wave' not in r['Kernel_Name']: continue
    tot[r['Counter_Name']] += float(r['Counter_Value']); disp.add(r.get('Dispatch_Id'))
nd = max(1, len(disp))
print(sys.argv[2], {k: round(v / nd / 1e6, 3) for k, v in tot.items()}, "M per dispatch,", nd, "dispatches")
PY
done
