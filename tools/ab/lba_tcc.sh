#!/bin/bash
# L2 hit rate and memory-side reads per LBA kernel (one PMC pass over one 128-window LBA call)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_lba_tcc
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_lba_tcc -o run -- python3 bench.py --legs lba --no-cpu-baseline --lba-calls 1 \
  > gpurun_out/pmc_lba_tcc.log 2>&1 || exit 1
python3 tools/lba_tcc.py gpurun_out/pmc_lba_tcc gpurun_out/lba_tcc.json | head -40
