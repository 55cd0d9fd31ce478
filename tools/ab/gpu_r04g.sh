#!/bin/bash
# round 4g evidence on the round's final LBA code: all GPU tests + smoke + default bench, the round
# profile (kernel stats, one batch in flight, PMC, LBA FP64), the drop-in kernel trace, then the
# batched LBA leg on the in-tree library and on a byte-identical copy, interleaved (run variance)
export TMPDIR=/tmp
bash tools/gpu_check.sh r04g || exit 1
SKIP_CAL=1 bash tools/profile_round.sh r04g > gpurun_out/profile_r04g.log 2>&1 || exit 1
bash tools/lba_dropin_prof.sh gpurun_out/dropin_r04g || exit 1
for i in 1 2 3; do
  for L in orb-slam3-noted_amd/lib/libslamhot.so orb-slam3-noted_amd/lib/ab/libslamhot_copy.so; do
    SLAMHOT_LIB=$L timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline > gpurun_out/lbav.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lbav.json'))['lba']; print('$(basename $L)', d['value'])"
  done
done
echo r04g_done
