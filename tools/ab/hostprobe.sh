nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; taskset -p $$; cat /proc/loadavg
python - <<'PY'
import sys
sys.path.insert(0,'orb-slam3-noted_amd'); sys.path.insert(0,'tests')
import shim_io
from slamhot import optimizer as opt, synth
W = synth.lba_window(0)
pmap,kfs,mps = opt.map_from_window(W)
shim_io.write_map('/tmp/lba_map.bin', pmap,kfs,mps)
PY
cat > /tmp/med.py <<'PY'
import numpy as np,sys; sys.path.insert(0,'tests'); import shim_io
b=shim_io.Blob(open(sys.argv[1],'rb').read()); v=b.vec('<f8'); print(sys.argv[2], 'median', np.round(np.median(v),3), 'min', np.round(v.min(),3))
PY
for i in 1 2; do for t in 1 2 4 8; do SLAMHOT_SHIM_THREADS=$t tests/cpp/shim_driver flattime /tmp/lba_map.bin /tmp/o.bin 40; python /tmp/med.py /tmp/o.bin flat$t; SLAMHOT_SHIM_THREADS=$t tests/cpp/shim_driver lbahost /tmp/lba_map.bin /tmp/o.bin 40; python /tmp/med.py /tmp/o.bin host$t; done; done
