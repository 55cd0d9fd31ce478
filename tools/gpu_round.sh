#!/bin/bash
# One GPU-box evidence run, parameterised (replaces the per-session gpu_rNNx.sh wrappers):
#   tools/gpu_round.sh TAG STEP [STEP ...]
# STEPs, run in order, the first failure ends the call:
#   check    all -m gpu tests + smoke() + the driver's bench command   (tools/gpu_check.sh)
#   tests    all -m gpu tests only
#   profile  rocprofv3 kernel traces + PMC of the round               (tools/profile_round.sh, SKIP_CAL=1)
#   dropin   kernel trace of LocalMapping's drop-in LBA call          (tools/lba_dropin_prof.sh)
#   launch2  bench.py --gpus 2 through its own launcher, both ranks on cuda:0 (gloo rehearsal of the
#            N-rank path on a one-GPU box), headline leg only
#   bench    the driver's exact bench command alone (tools/gpu_bench_driver.sh)
export TMPDIR=/tmp
TAG=$1
shift
mkdir -p gpurun_out
for step in "$@"; do
  echo "== $step ($TAG)"
  case $step in
    check)   bash tools/gpu_check.sh "$TAG" || exit 1 ;;
    profile) SKIP_CAL=1 bash tools/profile_round.sh "$TAG" > gpurun_out/profile_$TAG.log 2>&1 || exit 1 ;;
    dropin)  bash tools/lba_dropin_prof.sh gpurun_out/dropin_$TAG || exit 1 ;;
    launch2) SLAMHOT_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --legs headline --steps 20 \
               --warmup 3 --no-cpu-baseline > gpurun_out/launch2_$TAG.json 2> gpurun_out/launch2_$TAG.err || exit 1
             cat gpurun_out/launch2_$TAG.json ;;
    bench)   bash tools/gpu_bench_driver.sh "$TAG" || exit 1 ;;
    tests)   timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
               > gpurun_out/tests_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc ;;
    *)       echo "unknown step $step"; exit 2 ;;
  esac
done
echo "${TAG}_done"
