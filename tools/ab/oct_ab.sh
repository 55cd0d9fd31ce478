export TMPDIR=/tmp
T="tests/test_gpu_extractor.py tests/test_gpu_frame.py"
bash tools/ab/ab_env.sh oct "$T tests/test_gpu_stereo.py" headline,extract SLAMHOT_OCT_L0=0 SLAMHOT_OCT_L0=1 || exit 1
for v in 1 0; do SLAMHOT_OCT_SMALL=$v timeout -k 10 120 python3 tools/single_frame.py | sed "s/^/small=$v /" || exit 1; done
SLAMHOT_EXTRACT_GRAPH=0 SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_octr.so timeout -k 10 120 python3 tools/single_frame_trace.py > gpurun_out/octr.log 2>&1
