"""GPU: the kernels on the gate known-answer inputs (tests/gate_kats.py) decide as the compiled
reference's arithmetic does (and as the oracle does), where unfused float arithmetic would not."""
import numpy as np
import pytest

import gate_kats as G
import oracle_bind as ob
import scenes
from test_gate_kats import check_frustum, frustum_oracle, fuse_views, sbp_views

pytestmark = pytest.mark.gpu


def test_frustum_kats_gpu():
    import slamhot
    S, geom, limits, cases = G.frustum_cases(0)
    fv, keep = scenes.frame_view(S)
    desc = np.zeros((len(geom), 32), np.uint8)
    tr = np.zeros(len(geom), slamhot.MP_TRACK_DTYPE)
    m = slamhot.ORBmatcher(0.8)
    for lim in np.unique(limits):
        sel = np.flatnonzero(limits == lim)
        _, _, _, t = m.SearchLocalPoints(fv, geom[sel], desc[sel], 1.0, False, 50.0, float(lim))
        tr[sel] = t
    m.close()
    check_frustum(tr, cases)
    to = frustum_oracle(S, geom, limits)
    for f in ("in_view", "proj_x", "proj_y", "proj_xr", "depth", "view_cos", "scale_level"):
        assert np.array_equal(tr[f], to[f]), f


def test_triangulation_kats_gpu():
    import slamhot
    kfs, pairs, cases = G.triangulation_cases(0)
    m = slamhot.Mapper()
    res = m.SearchForTriangulation(kfs, pairs, False)
    m.close()
    for (n, mp), c in zip(res, cases):
        assert (n == 1) == c["fma"], c


def test_sbp_last_kats_gpu():
    import slamhot
    m = slamhot.ORBmatcher(0.9, False)
    for k in G.sbp_last_cases(0):
        fv, lf, keep = sbp_views(k)
        n, fm = m.SearchByProjection_last(fv, lf, float(k["th"]), False)
        assert (n == 1) == k["case"]["fma"], k
    m.close()


def test_fuse_kats_gpu():
    import slamhot
    m = slamhot.Mapper()
    for k in G.fuse_cases(0):
        fv, isg, g, d, keep = fuse_views(k)
        bi, bd = m.FuseSearch(fv, isg, g, d, 3.0)
        bo, do = ob.fuse_search(fv, isg, g, d, 3.0)
        assert (bd[0] == 0) == k["case"]["fma"] and bd[0] == do[0] and bi[0] == bo[0], k
    m.close()
