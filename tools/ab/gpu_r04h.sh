#!/bin/bash
# round 4h: the default bench line after bench.py's drop-in leg moved to 24 timed calls
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_r04h.json 2> gpurun_out/bench_r04h.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r04h.json'))
print('headline', d['value']); l=d['lba']; print('lba', l['value'], l['single_window']['drop_in'])"
