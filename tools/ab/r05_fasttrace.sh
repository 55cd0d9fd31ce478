#!/bin/bash
# k_fast_wave per-pass cycles and list sizes of sampled cells (SLAMHOT_FAST_TRACE build), frame 5
# of each headline batch, three headline steps; summary by level and attempt count.
export TMPDIR=/tmp
SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_ftrace.so timeout -k 10 200 python bench.py --legs headline --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/ftrace.json 2> gpurun_out/ftrace.err || exit 1
grep "^FAST lvl" gpurun_out/ftrace.json > gpurun_out/ftrace.txt
python3 - <<'PY'
import re, collections
rows = []
for l in open("gpurun_out/ftrace.txt"):
    d = dict(re.findall(r"(\w+)=(\d+)", l)); d.update({k: int(v) for k, v in re.findall(r" (zero|A|B1|B|C) (\d+)", l)})
    rows.append({k: int(v) for k, v in d.items()})
print("cells", len(rows))
by = collections.defaultdict(list)
for r in rows: by[(r["lvl"], r["att"])].append(r)
for k in sorted(by):
    v = by[k]; n = len(v)
    avg = lambda f: round(sum(r[f] for r in v) / n, 1)
    print(k, "n", n, "cw", avg("cw"), "ch", avg("ch"), "nA", avg("nA"), "nB1", avg("nB1"), "nB", avg("nB"), "kept", avg("kept"),
          "cyc zero", avg("zero"), "A", avg("A"), "B1", avg("B1"), "B", avg("B"), "C", avg("C"))
tot = collections.Counter()
for r in rows:
    for f in ("zero", "A", "B1", "B", "C"): tot[f] += r[f]
print("share", {f: round(tot[f] / sum(tot.values()), 3) for f in tot}, "att2 frac", round(sum(r["att"] == 2 for r in rows) / max(1, len(rows)), 3))
PY
