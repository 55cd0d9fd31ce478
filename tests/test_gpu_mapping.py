"""GPU parity: LocalMapping matchers vs the CPU oracle."""
import numpy as np
import pytest

import oracle_bind as ob
from test_mapping_oracle import observation_sets

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,max_n", [(1, 40), (2, 8), (3, 200)])
def test_distinctive_descriptors(seed, max_n):
    import slamhot
    off, desc = observation_sets(seed, 400 if max_n < 100 else 60, max_n)
    m = slamhot.Mapper()
    best = m.ComputeDistinctiveDescriptors(off, desc)
    assert np.array_equal(best, ob.distinctive_descriptors(off, desc))
    assert np.array_equal(m.ComputeDistinctiveDescriptors(np.zeros(1, np.int32), np.zeros((0, 32), np.uint8)),
                          np.zeros(0, np.int32))
    m.close()


@pytest.mark.parametrize("check_ori", [False, True])
def test_search_for_triangulation_batch(check_ori):
    """All neighbour pairs of KeyFrame 0 plus a few others in one launch, every flag
    combination, against the oracle pair by pair."""
    import scenes

    import slamhot
    kfs, poses = scenes.tri_keyframes(7, n_kf=5)
    pairs = []
    for a, b, only_stereo, coarse in [(0, 1, False, False), (0, 2, False, False), (0, 3, True, False),
                                      (0, 4, False, True), (2, 1, False, False), (4, 3, True, True),
                                      (1, 1, False, False)]:
        pairs.append((a, b, only_stereo, coarse))
    m = slamhot.Mapper()
    res = m.SearchForTriangulation(kfs, pairs, check_ori)
    m.close()
    built = [slamhot.make_tri_kf(k) for k in kfs]
    total = 0
    for (a, b, os_, co), (n, mp) in zip(pairs, res):
        no, m12 = ob.search_for_triangulation(built[a][0], built[b][0], slamhot.make_tri_pair(a, b, os_, co), check_ori)
        i1 = np.flatnonzero(m12 >= 0)
        assert n == no
        assert np.array_equal(mp, np.stack([i1, m12[i1]], 1))
        total += n
    assert total > 500


@pytest.mark.parametrize("seed,th", [(12, 3.0), (13, 1.0), (14, 5.0)])
def test_fuse_search(seed, th):
    import scenes

    import slamhot
    from slamhot import synth
    S = scenes.scene(seed)
    fv, keep = scenes.frame_view(S)
    geom, desc = scenes.fuse_mps(S)
    _, isig, _ = synth._level_tables()
    m = slamhot.Mapper()
    bi, bd = m.FuseSearch(fv, isig, geom, desc, th)
    m.close()
    bo, do = ob.fuse_search(fv, isig, geom, desc, th)
    assert np.array_equal(bi, bo)
    assert np.array_equal(bd, do)
    assert (bd <= 50).sum() > 100
