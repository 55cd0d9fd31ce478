"""GPU parity: device cv::remap(INTER_LINEAR) rectification vs the CPU oracle, bit-exact."""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob
from slamhot import euroc, synth

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden" / "euroc_stereo_calib.json"


def _maps(side):
    c = {k: np.array(v) if isinstance(v, list) else v for k, v in json.loads(GOLD.read_text()).items()}
    return euroc.init_undistort_rectify_map(c[f"{side}.K"], c[f"{side}.D"], c[f"{side}.R"], c[f"{side}.P"],
                                            (c[f"{side}.width"], c[f"{side}.height"]))


@pytest.mark.parametrize("side", ["LEFT", "RIGHT"])
def test_rectify_batch_bitexact(side):
    mx, my = _maps(side)
    imgs = np.stack([synth.frame(40 + i, 752, 480) for i in range(11)])
    r = euroc.Rectifier(mx, my)
    out = r(imgs)
    r.close()
    for i in (0, 5, 10):
        assert np.array_equal(out[i], ob.remap_linear(imgs[i], mx, my))


def test_rectify_borders_and_sizes():
    """Maps reaching outside the source (constant-0 border, partial 2x2 taps), exact half
    fractions, a destination narrower than a multiple of 4 and a smaller source."""
    rng = np.random.default_rng(1)
    dw, dh, sw, sh = 301, 97, 250, 90
    yy, xx = np.mgrid[0:dh, 0:dw].astype(np.float32)
    mx = (xx * 0.9 - 20 + rng.normal(0, 3, (dh, dw))).astype(np.float32)
    my = (yy * 1.05 - 5 + rng.normal(0, 2, (dh, dw))).astype(np.float32)
    mx[3, :50] = np.arange(50) + 0.015625
    src = rng.integers(0, 256, (3, sh, sw), dtype=np.uint8)
    r = euroc.Rectifier(mx, my, src_size=(sw, sh))
    out = r(src)
    r.close()
    for i in range(3):
        assert np.array_equal(out[i], ob.remap_linear(src[i], mx, my))
