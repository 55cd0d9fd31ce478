"""Regression against the committed fixtures (tests/golden/, made by tools/make_golden.py
from the oracle; inputs regenerate from seeds).  CPU: the oracle still reproduces them.
GPU: the HIP path reproduces them."""
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

G = Path(__file__).resolve().parent / "golden"
CASES = sorted(p.name for p in G.glob("extract_*.npz"))


def _load(name):
    z = np.load(G / name)
    img = synth.frame(int(z["seed"]), int(z["width"]), int(z["height"]))
    return z, img


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(name):
    z, img = _load(name)
    k, d, m = ob.extract(img, ob.params(nfeatures=int(z["nfeatures"])), lap=tuple(z["lap"]))
    assert m == int(z["mono"])
    assert np.array_equal(k.view(np.uint8), z["kps"].view(np.uint8))
    assert np.array_equal(d, z["desc"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_reproduces_golden(gpu_extractor_factory, name):
    z, img = _load(name)
    ex = gpu_extractor_factory(nfeatures=int(z["nfeatures"]), max_size=(int(z["width"]), int(z["height"])))
    k, d, m = ex(img, tuple(z["lap"]))
    assert m == int(z["mono"])
    assert np.array_equal(k.view(np.uint8), z["kps"].view(np.uint8))
    assert np.array_equal(d, z["desc"])


def test_oracle_bow_golden():
    z = np.load(G / "bow_pair.npz")
    img0 = synth.frame(1, 752, 480)
    img1 = synth.shifted(img0, 3, 2, 2.0, 7)
    k0, d0, _ = ob.extract(img0, ob.params(nfeatures=1200))
    k1, d1, _ = ob.extract(img1, ob.params(nfeatures=1200))
    A = (d0, k0["angle"], z["valid"]) + synth.feature_vector(z["node0"], z["w0"])
    B = (d1, k1["angle"], None) + synth.feature_vector(z["node1"], z["w1"])
    n, a2b, b2a = ob.search_by_bow(A, B, 0.7, True, False)
    assert n == int(z["nmatches"]) and np.array_equal(b2a, z["b2a"])
