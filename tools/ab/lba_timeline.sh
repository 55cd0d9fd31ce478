#!/bin/bash
# LBA leg: plan/device/wall split per call, and a kernel trace of the default 4-solver leg for
# the GPU-busy fraction (tools/busy.py).
export TMPDIR=/tmp
TAG=${1:-tl}
SLAMHOT_LBA_PLAN_TIMING=1 timeout -k 10 200 python tools/lba_bench.py --batches 1,128 --reps 3 > gpurun_out/lba_split_$TAG.log 2>&1 || exit 1
cat gpurun_out/lba_split_$TAG.log | tail -12
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lba_tl_$TAG -o t -- python3 bench.py --legs lba --no-cpu-baseline > gpurun_out/lba_tl_$TAG.json 2>gpurun_out/lba_tl_$TAG.err || exit 1
python3 tools/busy.py gpurun_out/lba_tl_$TAG
