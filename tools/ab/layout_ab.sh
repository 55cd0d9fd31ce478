#!/bin/bash
# k_layout A/B: parity tests per library, single-frame latency, then the headline / extract legs
export TMPDIR=/tmp
NEW=orb-slam3-noted_amd/lib/libslamhot.so; OLD=orb-slam3-noted_amd/lib/ab/libslamhot_lyold.so
for i in 1 2; do for L in $NEW $OLD; do SLAMHOT_LIB=$L timeout -k 10 120 python3 tools/single_frame.py | sed "s|^|$(basename $L) |" || exit 1; done; done
bash tools/ab/ab_var.sh ly "tests/test_gpu_extractor.py tests/test_gpu_frame.py tests/test_gpu_stereo.py" headline,extract $NEW $OLD
