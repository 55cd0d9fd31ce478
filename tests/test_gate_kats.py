"""The oracle on known-answer inputs that sit exactly on the contracted gates (tests/gate_kats.py):
it must decide as the compiled reference's arithmetic does, which is never what unfused float
arithmetic decides on these inputs."""
import numpy as np

import gate_kats as G
import oracle_bind as ob
import scenes
import slamhot


def frustum_oracle(S, geom, limits):
    fv, keep = scenes.frame_view(S)
    tr = np.zeros(len(geom), slamhot.MP_TRACK_DTYPE)
    for lim in np.unique(limits):
        sel = np.flatnonzero(limits == lim)
        _, t = ob.is_in_frustum(fv, geom[sel], float(lim))
        tr[sel] = t
    return tr


def check_frustum(tr, cases):
    for i, c in enumerate(cases):
        if c["kind"] == "level":
            assert tr["in_view"][i] == 1 and tr["scale_level"][i] == c["fma"], (i, c, tr[i])
        else:
            assert bool(tr["in_view"][i]) == c["fma"], (i, c, tr[i])


def test_frustum_kats_oracle():
    S, geom, limits, cases = G.frustum_cases(0)
    assert len(cases) >= 24
    check_frustum(frustum_oracle(S, geom, limits), cases)


def test_triangulation_kats_oracle():
    kfs, pairs, cases = G.triangulation_cases(0)
    assert len(cases) >= 16
    built = [slamhot.make_tri_kf(k) for k in kfs]
    for (a, b, os_, co), c in zip(pairs, cases):
        n, m12 = ob.search_for_triangulation(built[a][0], built[b][0], slamhot.make_tri_pair(a, b, os_, co), False)
        assert (n == 1) == c["fma"], c


def sbp_views(k):
    kp, d, ur = G._one_feature_frame(k["u"], k["v"], k["kpr"])
    fv, keep = slamhot.make_frame_view(kp, d, ur, np.full(1, -1, np.int8), Tcw=k["T"])
    lf, lkeep = slamhot.make_last_frame(k["T"], kp, kp, np.ones(1, np.uint8), np.zeros(1, np.uint8), k["X"][None],
                                        d, np.ones(1, np.uint8))
    return fv, lf, (keep, lkeep)


def test_sbp_last_kats_oracle():
    for k in G.sbp_last_cases(0):
        fv, lf, keep = sbp_views(k)
        n, fm = ob.search_by_projection_last(fv, lf, 0.9, False, float(k["th"]), False)
        assert (n == 1) == k["case"]["fma"], k


def fuse_views(k):
    kp, d, ur = G._one_feature_frame(k["kx"], k["ky"], k["kpr"])
    fv, keep = slamhot.make_frame_view(kp, d, ur, Tcw=np.eye(4, dtype=np.float32))
    isg = np.full(8, k["isg"], np.float32)
    return fv, isg, G.one_mp_geom(k["X"]), d, keep


def test_fuse_kats_oracle():
    for k in G.fuse_cases(0):
        fv, isg, g, d, keep = fuse_views(k)
        bi, bd = ob.fuse_search(fv, isg, g, d, 3.0)
        assert (bd[0] == 0) == k["case"]["fma"], (k, bi, bd)
