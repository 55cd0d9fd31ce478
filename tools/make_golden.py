"""Generate the committed regression fixtures in tests/golden/ from the CPU oracle.

The reference ships no golden vectors for this path and cannot be built here (SURVEY.md
§8c), so these fixtures pin the oracle restatement (and through the GPU tests the HIP path)
against regressions; they are NOT reference outputs.  Inputs are regenerated from seeds."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "orb-slam3-noted_amd")]
import numpy as np  # noqa: E402

import oracle_bind as ob  # noqa: E402
from slamhot import synth  # noqa: E402

OUT = ROOT / "tests" / "golden"


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    cases = [("vga_s0", 0, 640, 480, 1000, (0, 0)), ("euroc_s1", 1, 752, 480, 1200, (0, 0)),
             ("vga_s2_mono", 2, 640, 480, 1000, (0, 1000))]
    for name, seed, w, h, nf, lap in cases:
        img = synth.frame(seed, w, h)
        k, d, m = ob.extract(img, ob.params(nfeatures=nf), lap=lap)
        np.savez_compressed(OUT / f"extract_{name}.npz", seed=seed, width=w, height=h, nfeatures=nf,
                            lap=np.array(lap), kps=k, desc=d, mono=m)
    # SearchByBoW on a shifted pair with the synthetic k=10 L=6 vocabulary
    par, leaf, dn, wn = synth.vocab(10, 6, 0)
    img0 = synth.frame(1, 752, 480)
    img1 = synth.shifted(img0, 3, 2, 2.0, 7)
    k0, d0, _ = ob.extract(img0, ob.params(nfeatures=1200))
    k1, d1, _ = ob.extract(img1, ob.params(nfeatures=1200))
    _, w0, n0 = ob.vocab_transform(par, leaf, dn, wn, 6, d0, 4)
    _, w1, n1 = ob.vocab_transform(par, leaf, dn, wn, 6, d1, 4)
    valid = (np.random.default_rng(0).random(len(k0)) < 0.85).astype(np.uint8)
    A = (d0, k0["angle"], valid) + synth.feature_vector(n0, w0)
    B = (d1, k1["angle"], None) + synth.feature_vector(n1, w1)
    n, a2b, b2a = ob.search_by_bow(A, B, 0.7, True, False)
    np.savez_compressed(OUT / "bow_pair.npz", node0=n0, node1=n1, w0=w0, w1=w1, valid=valid, nmatches=n, b2a=b2a)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
