#!/bin/bash
# Experiment build of the product library with extra compile flags, for interleaved A/B runs on the
# GPU box:  tools/variant_lib.sh NAME "-DSLAMHOT_ST_CAND=8 ..."  ->  orb-slam3-noted_amd/lib/variant/NAME/libslamhot.so
# (git-ignored, travels with gpurun), selected at run time by SLAMHOT_LIB=<that path>.
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
FLAGS="$*"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result"
OBJ=build/variant/$NAME; OUT=orb-slam3-noted_amd/lib/variant/$NAME
mkdir -p $OBJ $OUT
ls orb-slam3-noted_amd/csrc/*.hip | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c -o $OBJ/\$(basename {} .hip).o {}"
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o $OUT/libslamhot.so $OBJ/*.o
echo "$OUT/libslamhot.so"
