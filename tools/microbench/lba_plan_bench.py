"""Experiment helper (CPU only): time the LBA host plan (plan_sizes + plan_fill) of a 128-window
config-4 call through an experiment library built with -DSLAMHOT_PLAN_BENCH:
    tools/build_variant.sh planbench -DSLAMHOT_PLAN_BENCH lba
    SLAMHOT_LBA_PLAN_THREADS=4 python tools/microbench/lba_plan_bench.py [windows] [reps]"""
import ctypes as C
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

nwin = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
L = C.CDLL(str(ROOT / "orb-slam3-noted_amd/lib/ab/libslamhot_planbench.so"))
pool = [synth.lba_window(s) for s in range(8)]
ws = [pool[i % len(pool)] for i in range(nwin)]
probs = (slamhot.LbaProblem * nwin)()
keep = []
for i, w in enumerate(ws):
    p, r, o = slamhot.make_lba_problem(w)
    probs[i] = p
    keep.append((p, r, o))
opt = slamhot.LbaOptions(5, 10, 0.0)
a, b, mb = C.c_double(), C.c_double(), C.c_double()
fn = L.slamhot_lba_plan_bench
fn.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
t0 = time.perf_counter()
st = fn(nwin, C.addressof(probs), C.addressof(opt), reps, C.byref(a), C.byref(b), C.byref(mb))
dt = (time.perf_counter() - t0) / reps * 1e3
print(f"status {st} windows {nwin} sizes {a.value:.3f} ms fill {b.value:.3f} ms arena {mb.value:.1f} MB (wall/rep {dt:.2f} ms)")
