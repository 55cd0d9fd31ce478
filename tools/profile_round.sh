#!/bin/bash
# Round profile evidence (run on the GPU box from the repo root):
#   0. FETCH_SIZE calibration (tools/microbench/mb_fetch, built on the CPU beforehand)
#   1. rocprofv3 --kernel-trace --stats of the default bench      -> gpurun_out/prof_default/
#   2. the headline leg alone with one batch in flight               -> gpurun_out/prof_inflight1/
#      (its k_fast_wave average is what bench.py reports as roofline.avg_launch_ms)
#   3. PMC passes (--pmc only) over the same run -> profiles/traffic_latest.json
#   4. PMC pass over the LBA leg (MFMA busy cycles)                 -> gpurun_out/pmc_lba/
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r02}
if [ -z "$SKIP_CAL" ]; then  # SKIP_CAL=1: keep the committed profiles/fetch_calibration.json
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
  -- tools/microbench/mb_fetch > gpurun_out/pmc_fetch.log 2>&1
python3 tools/fetch_calibrate.py gpurun_out/pmc_fetch
fi
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run \
  -- python3 bench.py --in-process > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inflight1 -o run \
  -- python3 bench.py --in-process --inflight 1 --no-cpu-baseline --legs headline \
  > gpurun_out/prof_inflight1.json 2> gpurun_out/prof_inflight1.err
SLAMHOT_SERIAL=1 bash tools/profile_counters.sh gpurun_out/pmc --in-process --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 \
  --legs headline > gpurun_out/pmc.log 2>&1
python3 tools/parse_counters.py gpurun_out/pmc k_fast_wave 256 752 2 > /dev/null
mkdir -p gpurun_out/pmc_lba
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_lba/p1 -o run -- python3 bench.py --in-process --legs lba --no-cpu-baseline --lba-calls 1 \
  > gpurun_out/pmc_lba.log 2>&1
python3 tools/parse_counters.py gpurun_out/pmc_lba > /dev/null
find gpurun_out/prof_default gpurun_out/prof_inflight1 -name "*kernel_stats.csv"
