#!/bin/bash
# k_fast_wave / k_orb3 issue counters per wave, in-tree library vs lib/ab/libslamhot_head.so (one
# rocprofv3 --pmc pass each, headline leg, one batch in flight).  Usage: r05_fastpmc.sh TAG
export TMPDIR=/tmp
TAG=${1:-fastpmc}
A=orb-slam3-noted_amd/lib/libslamhot.so; B=${HEADLIB:-orb-slam3-noted_amd/lib/ab/libslamhot_head.so}
for L in $A $B; do
  n=$(basename $L .so)
  SLAMHOT_LIB=$L timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d gpurun_out/${TAG}_pmc/$n -o run -- python3 bench.py --legs headline --inflight 1 --no-cpu-baseline --steps 5 --warmup 1 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/${TAG}_pmc/$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections, os
for kern in ("k_fast_wave", "k_orb3"):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(sys.argv[1])):
        if kern in r["Kernel_Name"]: acc[r["Counter_Name"]] += float(r["Counter_Value"])
    st = [r for r in csv.DictReader(open(os.path.join(os.path.dirname(sys.argv[1]), "run_kernel_stats.csv"))) if kern in r["Name"]]
    w = max(1.0, acc["SQ_WAVES"])
    print(sys.argv[2], kern, "waves", round(w), "per wave: valu", round(acc["SQ_INSTS_VALU"] / w, 1), "salu", round(acc["SQ_INSTS_SALU"] / w, 1),
          "lds", round(acc["SQ_INSTS_LDS"] / w, 1), "active_valu", round(acc["SQ_ACTIVE_INST_VALU"] / w, 1), "lds_conflict", round(acc["SQ_LDS_BANK_CONFLICT"] / w, 1),
          "wave_cycles", round(4 * acc["SQ_WAVE_CYCLES"] / w), "avg us", round(float(st[0]["AverageNs"]) / 1e3, 1) if st else None)
PY
done
