#!/bin/bash
# k_octree phase cycles per (frame, level) (SLAMHOT_OCTREE_TRACE build), one wave per (frame, level)
# vs SLAMHOT_OCT_L0=1 SLAMHOT_OCT_REST=1 (4 waves)
export TMPDIR=/tmp
for cfg in "0 0"; do
  set -- $cfg
  SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_octtrace.so SLAMHOT_OCT_L0=$1 SLAMHOT_OCT_REST=$2 timeout -k 10 200 python bench.py --legs headline --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/octtrace_$1$2.json 2> gpurun_out/octtrace_$1$2.err || exit 1
  grep "^OCT W" gpurun_out/octtrace_$1$2.json | head -400 > gpurun_out/octtrace_$1$2.txt
  python3 - gpurun_out/octtrace_$1$2.txt "L0=$1 REST=$2" <<'PY'
import re, sys, collections
by = collections.defaultdict(list)
for l in open(sys.argv[1]):
    m = re.match(r"OCT W=(\d+) f=(\d+) l=(\d+) nk=(\d+) n=(\d+) marks=(\d+): ([\d\- ]+) tot=(\d+)", l)
    if not m: continue
    W, f, lv, nk, n, marks = map(int, m.groups()[:6]); d = list(map(int, m.group(7).split())); tot = int(m.group(8))
    by[lv].append((W, nk, n, marks, d, tot))
print(sys.argv[2])
for lv in sorted(by):
    v = by[lv]; k = len(v)
    avg = lambda i: round(sum(x[4][i] for x in v) / k)
    print(" l", lv, "W", v[0][0], "nk", round(sum(x[1] for x in v) / k), "passes", v[0][3] - 3, "gather", avg(0), "init", avg(1),
          "pass1..", [avg(i) for i in range(2, min(9, v[0][3] - 1))], "tot", round(sum(x[5] for x in v) / k))
PY
done
