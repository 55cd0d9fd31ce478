export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_frame.py tests/test_gpu_cpp_host.py tests/test_gpu_stereo.py tests/test_gpu_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sb_tests.log 2>&1; echo sb_tests=$?; tail -1 gpurun_out/sb_tests.log
timeout -k 10 120 python3 tools/single_frame.py
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_sf2 -o run -- python3 tools/single_frame.py > gpurun_out/sf2.log 2>&1; echo rc=$?
timeout -k 10 200 python bench.py --legs extract,track --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/sb.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/sb.json')); print(d['extract']['value'], d['extract']['host_path'], d['track']['value'], d['track']['single_sequence'])"
