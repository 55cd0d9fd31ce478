#!/bin/bash
# k_orb3 per-phase cycles (SLAMHOT_ORB_TRACE build: s_memtime marks of sampled keypoints of frame 100)
export TMPDIR=/tmp
SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_orbtrace.so timeout -k 10 200 python bench.py --legs headline --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/orbtrace.json 2> gpurun_out/orbtrace.err
rc=$?; grep "ORB slot" gpurun_out/orbtrace.err | head -400 > gpurun_out/orbtrace.txt; wc -l gpurun_out/orbtrace.txt
python3 - <<'PY'
import re, collections
tot = collections.defaultdict(list)
for l in open("gpurun_out/orbtrace.txt"):
    m = re.search(r"l=(\d+) stage (\d+) ic (\d+) horiz (\d+) sincos (\d+) desc (\d+)", l)
    if m:
        for k, v in zip(("stage", "ic", "horiz", "sincos", "desc"), m.groups()[1:]):
            tot[k].append(int(v))
for k, v in tot.items():
    v.sort(); print(k, "n", len(v), "median", v[len(v) // 2], "mean", sum(v) / len(v))
PY
exit $rc
