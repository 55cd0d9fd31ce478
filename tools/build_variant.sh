#!/bin/bash
# Experiment library: extractor.hip (or FILE) rebuilt with extra flags, linked with the other
# in-tree objects.  Usage: tools/build_variant.sh NAME "FLAGS" [FILE]  -> lib/ab/libslamhot_NAME.so
set -e
NAME=$1; FLAGS=$2; FILE=${3:-extractor}
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result"
mkdir -p build/ab orb-slam3-noted_amd/lib/ab
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c -o build/ab/${FILE}_$NAME.o orb-slam3-noted_amd/csrc/$FILE.hip
OBJS=$(ls build/obj/*.o | grep -v "/$FILE.o")
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o orb-slam3-noted_amd/lib/ab/libslamhot_$NAME.so build/ab/${FILE}_$NAME.o $OBJS
echo built orb-slam3-noted_amd/lib/ab/libslamhot_$NAME.so
