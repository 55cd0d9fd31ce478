#!/bin/bash
# The driver's exact bench command, timed as the driver times it (wall seconds in the .wall file).
export TMPDIR=/tmp
TAG=${1:-d}
mkdir -p gpurun_out
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
t1=$(date +%s.%N)
python3 -c "print(f'bench_wall_s={$t1-$t0:.1f} rc=$rc')" | tee gpurun_out/bench_$TAG.wall
grep "bench\[" gpurun_out/bench_$TAG.err | tail -40
[ $rc -ne 0 ] && exit $rc
cat gpurun_out/bench_$TAG.json
