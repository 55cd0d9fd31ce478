"""LBA drop-in latency probe (GPU box): one config-4 window through tests/cpp/shim_driver lbatime,
with the phase split (window build + flatten / solve / rest) and the solver's own stats.
usage: python tools/lba_dropin.py [reps] [--write-map PATH]"""
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import shim_io  # noqa: E402
from slamhot import optimizer as opt  # noqa: E402
from slamhot import synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 12
    W = synth.lba_window(0)
    pmap, kfs, mps = opt.map_from_window(W)
    d = Path(tempfile.mkdtemp())
    mp, op = d / "map.bin", d / "out.bin"
    shim_io.write_map(mp, pmap, kfs, mps)
    if "--write-map" in sys.argv:
        import shutil
        shutil.copy(mp, sys.argv[sys.argv.index("--write-map") + 1])
    r = subprocess.run([str(shim_io.DRIVER), "lbatime", str(mp), str(op), str(reps)], capture_output=True, text=True,
                       timeout=300)
    print(r.stderr[-2000:])
    b = shim_io.Blob(op.read_bytes())
    counts = [b.i32() for _ in range(4)]
    ms, st, bld, sol = b.vec("<f8"), b.vec("<f8"), b.vec("<f8"), b.vec("<f8")
    print("counts", counts)
    print("call ms", np.round(ms, 3))
    print(f"median call {np.median(ms[1:]):.3f} ms; first {ms[0]:.3f} ms")
    print(f"build+flatten median {np.median(bld):.3f} ms; solve median {np.median(sol):.3f} ms")
    print(f"device {st[0]:.3f} ms, plan {st[1]:.3f} ms, syncs {int(st[2])}")


if __name__ == "__main__":
    main()
