#!/bin/bash
# Copy one evidence run (tools/gpu_check.sh TAG && tools/profile_round.sh TAG) from gpurun_out/
# into profiles/TAG_*, recomputing the PMC summaries locally.  Usage: tools/save_profiles.sh TAG
set -e
T=$1
python3 tools/parse_counters.py gpurun_out/pmc k_fast_wave 256 752 2 > /dev/null
python3 tools/lba_pmc.py gpurun_out/pmc_lba $T > /dev/null
cp gpurun_out/bench_$T.json profiles/${T}_bench.json
cp gpurun_out/prof_default.json profiles/${T}_bench_under_rocprof.json
cp gpurun_out/prof_inflight1.json profiles/${T}_inflight1_bench.json
cp gpurun_out/prof_default/run_kernel_stats.csv profiles/${T}_default_kernel_stats.csv
cp gpurun_out/prof_inflight1/run_kernel_stats.csv profiles/${T}_inflight1_kernel_stats.csv
cp gpurun_out/pmc/summary.json profiles/${T}_pmc_summary.json
grep -v amdgpu.ids gpurun_out/tests_$T.log | tail -4 > profiles/${T}_gpu_tests.log
ls profiles/${T}_*
