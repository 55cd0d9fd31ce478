#!/bin/bash
# k_ldlt_t16 with 16 / 12 / 8 waves per workgroup (mb_ldlt, n = 288 and 192), interleaved twice
export TMPDIR=/tmp
cd tools/microbench
for r in 1 2; do for b in mb_ldlt mb_ldlt_w12 mb_ldlt_w8; do
  echo -n "$b "; timeout -k 10 60 ./$b | grep t16 | cut -c1-40 | tr '\n' ' '; timeout -k 10 60 ./$b 192 | grep t16 | cut -c1-40 || exit 1
done; done
