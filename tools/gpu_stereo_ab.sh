# k_stereo_match with the packed band table: stereo / frame / shim / track GPU tests, the headline
# leg twice, and the kernel stats of one --inflight 1 headline run.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stereo.py tests/test_gpu_frame.py tests/test_gpu_shim.py tests/test_gpu_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/st_tests.log 2>&1 || { tail -30 gpurun_out/st_tests.log; exit 1; }
tail -2 gpurun_out/st_tests.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --legs headline --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/st_head$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/st_head$i.json')); print('headline', d['value'], d['ms_per_step'], d['headline_detail']['stage_ms_per_step'])"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_prof -o run \
  -- python3 bench.py --in-process --inflight 1 --legs headline --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/st_prof.json 2> gpurun_out/st_prof.err || exit 1
f=$(find gpurun_out/st_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/st_kernel_stats.csv && grep -E "stereo|remap" gpurun_out/st_kernel_stats.csv | cut -c1-200 || true
