#!/bin/bash
# round 4j evidence on the final tree (LDL^T spare-SIMD panels, PoseOptimization leg on prepared frames): all GPU tests +
# smoke + default bench, the round profile, the drop-in kernel trace
export TMPDIR=/tmp
bash tools/gpu_check.sh r04j || exit 1
SKIP_CAL=1 bash tools/profile_round.sh r04j > gpurun_out/profile_r04j.log 2>&1 || exit 1
bash tools/lba_dropin_prof.sh gpurun_out/dropin_r04j || exit 1
echo r04j_done
