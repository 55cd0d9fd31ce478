#!/bin/bash
# Experiment library of the last commit's FILE (default extractor) linked with the in-tree objects
# of the other files: lib/ab/libslamhot_NAME.so (default head), the baseline of tools/ab/r05_vs_head.sh.
set -e
FILE=${1:-extractor}
NAME=${2:-head}
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result"
mkdir -p build/ab orb-slam3-noted_amd/lib/ab
git show HEAD:orb-slam3-noted_amd/csrc/$FILE.hip > orb-slam3-noted_amd/csrc/zz_head_$FILE.hip
trap 'rm -f orb-slam3-noted_amd/csrc/zz_head_$FILE.hip' EXIT
/opt/rocm/bin/hipcc $HIPFLAGS -c -o build/ab/${FILE}_head.o orb-slam3-noted_amd/csrc/zz_head_$FILE.hip
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o orb-slam3-noted_amd/lib/ab/libslamhot_$NAME.so build/ab/${FILE}_head.o $(ls build/obj/*.o | grep -v "/$FILE.o")
echo built orb-slam3-noted_amd/lib/ab/libslamhot_$NAME.so
