#!/bin/bash
# Drop-in LocalBundleAdjustment latency (GPU box): the shim's host phases and the solver's phase
# trace, then releaser on / inline interleaved.  Usage: tools/lba_dropin_ab.sh
export TMPDIR=/tmp
SLAMHOT_LBA_TRACE=1 timeout -k 10 100 python tools/lba_dropin.py 6 || exit 1
for i in 1 2 3; do
  echo "== releaser thread"; timeout -k 10 100 python tools/lba_dropin.py 16 | grep -E 'median|device' || exit 1
  echo "== inline release"; SLAMHOT_RELEASE_INLINE=1 timeout -k 10 100 python tools/lba_dropin.py 16 | grep -E 'median|device' || exit 1
done
