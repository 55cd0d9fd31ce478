export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py tests/test_gpu_cpp_host.py tests/test_gpu_shim.py tests/test_gpu_stereo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hg_tests.log 2>&1; echo hg_tests=$?; tail -1 gpurun_out/hg_tests.log
for E in SLAMHOT_EXTRACT_GRAPH=0 SLAMHOT_EXTRACT_GRAPH=1; do
  env $E timeout -k 10 200 python bench.py --legs extract --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/hg_$E.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/hg_$E.json')); print('$E', d['extract']['host_path'])"
done
SLAMHOT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --legs headline,extract,lba > gpurun_out/tr2.json 2> gpurun_out/tr2.err; echo tr2=$?
python3 -c "
import json; d=json.load(open('gpurun_out/tr2.json')); print(d['n_gpus'], d['value'], d['headline_detail']['rank_digests'], d['extract']['value'], d['lba']['value'])"
