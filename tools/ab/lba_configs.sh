set -e
export SLAMHOT_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --legs headline,extract,lba,pose,track,localmap --track-frames 16 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
unset SLAMHOT_BENCH_BACKEND
for cfg in "64 3" "128 3" "64 6" "128 4" "256 2"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --legs lba --no-cpu-baseline --lba-windows $1 --lba-inflight $2 > gpurun_out/lba_$1_$2.json 2>/dev/null
done
