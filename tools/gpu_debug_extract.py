"""Stage-by-stage comparison of the GPU extractor against the oracle (debug aid)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam3-noted_amd"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import oracle_bind as ob  # noqa: E402
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402


def main():
    for (w, h) in [(640, 480), (752, 480), (1280, 720)]:
        img = synth.frame(1, w, h)
        ex = slamhot.ORBextractor(nfeatures=1000, max_size=(w, h))
        kg, dg, mg = ex(img)
        ko, do, mo = ob.extract(img)
        pyr = ob.pyramid(img)
        pyr_ok = [bool(np.array_equal(ex.pyramid_level(l), pyr[l])) for l in range(8)]
        print(f"{w}x{h}: pyramid {pyr_ok}")
        ko2, counts = ob.keypoints_octree(img)
        print(f"  n gpu {len(kg)} oracle {len(ko)} mono {mg}/{mo}; oracle per-level {counts.tolist()}")
        gl = np.bincount(kg["octave"], minlength=8)
        print(f"  gpu per-level {gl.tolist()}")
        if len(kg) == len(ko):
            for f in ("x", "y", "response", "octave", "angle", "size"):
                print(f"  field {f} mismatches {(kg[f] != ko[f]).sum()}")
            print(f"  desc mismatches {(dg != do).any(axis=1).sum()}")
        else:
            for l in range(8):
                a = kg[kg["octave"] == l]
                b = ko[ko["octave"] == l]
                sa = set(zip(a["x"].tolist(), a["y"].tolist()))
                sb = set(zip(b["x"].tolist(), b["y"].tolist()))
                print(f"  level {l}: gpu {len(a)} oracle {len(b)} common {len(sa & sb)}")
        ex.close()


if __name__ == "__main__":
    main()
