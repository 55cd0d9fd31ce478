#!/bin/bash
# round 4i evidence on the final tree (bench default now four batches in flight): all GPU tests +
# smoke + default bench, the round profile, the drop-in kernel trace
export TMPDIR=/tmp
bash tools/gpu_check.sh r04i || exit 1
SKIP_CAL=1 bash tools/profile_round.sh r04i > gpurun_out/profile_r04i.log 2>&1 || exit 1
bash tools/lba_dropin_prof.sh gpurun_out/dropin_r04i || exit 1
echo r04i_done
