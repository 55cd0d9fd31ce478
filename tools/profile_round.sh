#!/bin/bash
# Round profile evidence (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the default bench      -> gpurun_out/prof_default/
#   2. the same with one extraction batch in flight, other legs off -> gpurun_out/prof_inflight1/
#      (its k_fast_wave average is what bench.py reports as roofline.avg_launch_ms)
#   3. PMC passes (--pmc only, kernel-trace implied) for HBM bytes -> profiles/traffic_latest.json
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run \
  -- python3 bench.py > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inflight1 -o run \
  -- python3 bench.py --inflight 1 --no-cpu-baseline --match-pairs 0 --lba-windows 0 --pose-frames 0 --stereo-pairs 0 \
  > gpurun_out/prof_inflight1.json 2> gpurun_out/prof_inflight1.err
SLAMHOT_SERIAL=1 bash tools/profile_counters.sh gpurun_out/pmc --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 \
  --match-pairs 0 --lba-windows 0 --pose-frames 0 --stereo-pairs 0 > gpurun_out/pmc.log 2>&1
python3 tools/parse_counters.py gpurun_out/pmc k_fast_wave 256 640 > /dev/null
find gpurun_out/prof_default gpurun_out/prof_inflight1 -name "*kernel_stats.csv"
