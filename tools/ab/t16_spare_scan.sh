#!/bin/bash
# k_ldlt_t16 spare-SIMD threshold scan in mb_ldlt (n = 288 and 192), interleaved three times
export TMPDIR=/tmp
cd tools/microbench
for r in 1 2 3; do for v in 0 16 32 48 64 80; do
  echo -n "spare $v "; timeout -k 10 60 ./mb_ldlt_sp$v | grep t16 | cut -c1-30 | tr '\n' ' '; timeout -k 10 60 ./mb_ldlt_sp$v 192 | grep t16 | cut -c1-30 || exit 1
done; done
