#!/bin/bash
# One GPU call for a round's evidence: GPU tests + smoke + default bench line (tools/gpu_check.sh),
# then tools/profile_round.sh steps 1-4 (kernel stats, one-batch-in-flight headline, PMC passes,
# LBA FP64 / MFMA counters).  FETCH_SIZE calibration (step 0) is profiles/fetch_calibration.json.
TAG=${1:-r02f}
bash tools/gpu_check.sh $TAG || exit 1
export TMPDIR=/tmp
set -e
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run \
  -- python3 bench.py --in-process > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inflight1 -o run \
  -- python3 bench.py --in-process --inflight 1 --no-cpu-baseline --legs headline \
  > gpurun_out/prof_inflight1.json 2> gpurun_out/prof_inflight1.err
SLAMHOT_SERIAL=1 bash tools/profile_counters.sh gpurun_out/pmc --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 \
  --legs headline > gpurun_out/pmc.log 2>&1
python3 tools/parse_counters.py gpurun_out/pmc k_fast_wave 256 752 2 > /dev/null
mkdir -p gpurun_out/pmc_lba
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_lba/p1 -o run -- python3 bench.py --in-process --legs lba --no-cpu-baseline --lba-calls 1 \
  > gpurun_out/pmc_lba.log 2>&1
python3 tools/parse_counters.py gpurun_out/pmc_lba > /dev/null
find gpurun_out/prof_default gpurun_out/prof_inflight1 -name "*kernel_stats.csv"
echo evidence_done
