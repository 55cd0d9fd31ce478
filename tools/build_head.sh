#!/bin/bash
# Experiment library of the last commit's FILES (default extractor; several: "extractor matcher")
# linked with the in-tree objects of the other files: lib/ab/libslamhot_NAME.so (default head), the
# baseline of tools/ab/r05_vs_head.sh.
set -e
FILES=${1:-extractor}
NAME=${2:-head}
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result"
mkdir -p build/ab orb-slam3-noted_amd/lib/ab
OBJS=$(ls build/obj/*.o)
HOBJS=""
for FILE in $FILES; do
  git show HEAD:orb-slam3-noted_amd/csrc/$FILE.hip > orb-slam3-noted_amd/csrc/zz_head_$FILE.hip
  /opt/rocm/bin/hipcc $HIPFLAGS -c -o build/ab/${FILE}_head.o orb-slam3-noted_amd/csrc/zz_head_$FILE.hip || { rm -f orb-slam3-noted_amd/csrc/zz_head_$FILE.hip; exit 1; }
  rm -f orb-slam3-noted_amd/csrc/zz_head_$FILE.hip
  OBJS=$(echo "$OBJS" | grep -v "/$FILE.o")
  HOBJS="$HOBJS build/ab/${FILE}_head.o"
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o orb-slam3-noted_amd/lib/ab/libslamhot_$NAME.so $HOBJS $OBJS
echo built orb-slam3-noted_amd/lib/ab/libslamhot_$NAME.so
