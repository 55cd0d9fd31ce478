#!/bin/bash
# k_ldlt_reg (tiles resident in VGPRs, SLAMHOT_LDLT=reg) vs k_ldlt_t16: bitwise agreement and
# time in mb_ldlt at three sizes, LBA parity with reg forced, isolated kernel stats, the
# drop-in call and the LBA leg, interleaved
export TMPDIR=/tmp
for n in 288 192 100; do (cd tools/microbench && timeout -k 10 60 ./mb_ldlt $n | grep -E "t16|reg") || exit 1; done
SLAMHOT_LDLT=reg timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py tests/test_gpu_shim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ldlt_reg_tests.log 2>&1
rc=$?; echo "reg tests rc=$rc: $(tail -1 gpurun_out/ldlt_reg_tests.log)"; [ $rc -ne 0 ] && exit $rc
for v in t16 reg; do
  SLAMHOT_LDLT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ldlt_$v -o run -- python3 bench.py --legs lba --no-cpu-baseline --lba-inflight 1 --lba-calls 2 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/prof_ldlt_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:4]: print(r['Name'][:40].ljust(40), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
done
for i in 1 2; do
  for v in t16 reg; do
    echo -n "$v drop-in: "; SLAMHOT_LDLT=$v timeout -k 10 100 python tools/lba_dropin.py 24 2>&1 | grep -E "median call|device" | tr '\n' ' '; echo
    SLAMHOT_LDLT=$v timeout -k 10 300 python bench.py --legs lba --no-cpu-baseline > gpurun_out/lbar.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lbar.json'))['lba']; print('$v leg', d['value'], d['single_window']['ms_per_lm_iteration'])"
  done
done
