# LBA leg over calls per solver / solvers in flight / stagger (bench.py --legs lba), in the order given:
#   tools/gpu_lba_sweep.sh "CALLS INFLIGHT STAGGER_MS" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --legs lba --no-cpu-baseline --lba-calls $1 --lba-inflight $2 --lba-stagger-ms $3 > gpurun_out/lba_$1_$2_$3.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/lba_$1_$2_$3.json')); l=d.get('lba', d); print('calls $1 inflight $2 stagger $3', l['value'], l.get('ms_per_call'), l.get('host_plan_ms_per_call'))"
done
