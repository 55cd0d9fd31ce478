# k_update with Hpl recomputed (default) vs read back (SLAMHOT_UPD_RECOMPUTE=0 build, lib/ab/libslamhot_updread.so):
# LBA-side GPU tests, bitwise comparison of 12 solved windows, kernel stats of the LBA leg under each.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lba.py tests/test_gpu_pose.py tests/test_gpu_track.py tests/test_gpu_shim.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread > gpurun_out/upd_tests.log 2>&1 || { tail -20 gpurun_out/upd_tests.log; exit 1; }
tail -1 gpurun_out/upd_tests.log
timeout -k 10 200 python3 tools/lba_bits.py gpurun_out/bits_new.npz || exit 1
SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_updread.so timeout -k 10 200 python3 tools/lba_bits.py gpurun_out/bits_old.npz || exit 1
python3 -c "
import numpy as np
a, b = np.load('gpurun_out/bits_new.npz'), np.load('gpurun_out/bits_old.npz')
bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
print('bitwise identical' if not bad else 'DIFFERS: ' + ', '.join(bad[:10]), len(a.files), 'arrays')"
for v in new old; do
  if [ $v = old ]; then export SLAMHOT_LIB=orb-slam3-noted_amd/lib/ab/libslamhot_updread.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/upd_prof_$v -o run \
    -- python3 bench.py --in-process --legs lba --no-cpu-baseline > gpurun_out/upd_$v.json 2> gpurun_out/upd_$v.err || exit 1
  f=$(find gpurun_out/upd_prof_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "k_update|k_linearize|k_schur_rows" "$f" | awk -F',' '{print $1, $2, $(NF-4)}' | cut -c1-120
  python3 -c "import json; d=json.load(open('gpurun_out/upd_$v.json')); l=d.get('lba', d); print('$v LBA', l['value'])"
done
