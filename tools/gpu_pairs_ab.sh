export TMPDIR=/tmp
for cfg in "128 4" "256 4" "128 4" "256 4" "256 3" "256 5" "384 4"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --legs headline --steps 20 --warmup 5 --pairs $1 --inflight $2 --no-cpu-baseline > gpurun_out/pairs_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/pairs_$1_$2.json')); print('pairs $1 inflight $2', d['value'], d['ms_per_step'])"
done
