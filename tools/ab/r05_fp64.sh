export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_pose.py tests/test_gpu_track.py tests/test_gpu_shim.py tests/test_gpu_cpp_host.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_r05b.log 2>&1
rc=$?; tail -5 gpurun_out/tests_r05b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --legs lba,pose,track --no-cpu-baseline > gpurun_out/bench_r05b.json 2> gpurun_out/bench_r05b.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_r05b.json'))
print('lba', d['lba']['value'], d['lba']['single_window']['drop_in']['wall_ms_per_call'], 'pose', d['pose']['value'], 'track', d['track']['value'])"
