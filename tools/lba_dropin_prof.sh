#!/bin/bash
# Kernel trace of the single-window drop-in LocalBundleAdjustment call (GPU box):
# tools/lba_dropin_prof.sh OUTDIR
set -e
out=${1:-gpurun_out/lba_dropin_prof}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/lba_dropin.py 3 --write-map /tmp/lba_map.bin > "$out/probe.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out" -o lba -- tests/cpp/shim_driver lbatime /tmp/lba_map.bin /tmp/lba_out.bin 12 > "$out/rocprof.log" 2>&1
