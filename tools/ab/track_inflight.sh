#!/bin/bash
# track leg: the 64 sequences on 1 / 2 / 4 tracker handles (own streams), interleaved twice
export TMPDIR=/tmp
for r in 1 2; do
  for g in 1 2 4; do
    timeout -k 10 300 python bench.py --legs track --no-cpu-baseline --track-inflight $g > gpurun_out/trk.json 2>gpurun_out/trk.err || { tail -5 gpurun_out/trk.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/trk.json'))['track']; print('handles $g', d['value'], d['ms_per_step'], 'lost', d['lost_frames'], 'kfs', d['keyframes'], 'ate', d['ate_seq0_m'])"
  done
done
