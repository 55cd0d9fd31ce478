"""GPU parity: vocabulary descent and SearchByBoW (both variants) vs the CPU oracle."""
import numpy as np
import pytest

import oracle_bind as ob
from slamhot import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vocab_arrays():
    return synth.vocab(10, 6, 0)


@pytest.fixture(scope="module")
def gpu_vocab(vocab_arrays):
    import slamhot
    par, leaf, d, w = vocab_arrays
    v = slamhot.Vocabulary(par, leaf, d, w, k=10, L=6)
    yield v
    v.close()


@pytest.fixture(scope="module")
def frames():
    img0 = synth.frame(1, 752, 480)
    out = []
    for i, (dx, dy, a) in enumerate([(0, 0, 0), (3, 2, 2.0), (-4, 5, -4.0), (6, -3, 9.0)]):
        img = img0 if i == 0 else synth.shifted(img0, dx, dy, a, 7 + i)
        k, d, _ = ob.extract(img, ob.params(nfeatures=1200))
        out.append((k, d))
    return out


def test_vocab_transform_bitexact(gpu_vocab, vocab_arrays, frames):
    par, leaf, d, w = vocab_arrays
    for levelsup in (4, 2, 6, 0):
        for k, desc in frames:
            wg, wtg, ng = gpu_vocab.transform(desc, levelsup)
            wo, wto, no = ob.vocab_transform(par, leaf, d, w, 6, desc, levelsup)
            assert np.array_equal(wg, wo)
            assert np.array_equal(wtg, wto)
            assert np.array_equal(ng, no)


@pytest.mark.parametrize("k,L", [(20, 3), (17, 3), (16, 4), (3, 6), (5, 1)])
def test_vocab_transform_branching(k, L):
    """Branching factors around the kernel's register-held child slots (16 per node): k > 16
    takes the spill loop and reads the winner's record from memory, k <= 16 gets it from the
    winning lane; L = 1 stops at the root's children.  Same words / weights / nodes as the
    oracle descent (TemplatedVocabulary.h:1229-1271) at every levelsup."""
    import slamhot
    par, leaf, d, w = synth.vocab(k, L, 5)
    v = slamhot.Vocabulary(par, leaf, d, w, k=k, L=L)
    _, desc, _ = ob.extract(synth.frame(78, 640, 480))
    for levelsup in sorted({0, 1, L}):
        got = v.transform(desc, levelsup)
        ref = ob.vocab_transform(par, leaf, d, w, L, desc, levelsup)
        for x, y in zip(got, ref):
            assert np.array_equal(x, y), (k, L, levelsup)
    v.close()


def _side(gpu_vocab, k, desc, valid):
    _, wt, nid = gpu_vocab.transform(desc, 4)
    return (desc, k["angle"], valid) + synth.feature_vector(nid, wt)


@pytest.mark.parametrize("nnratio,check_ori", [(0.7, True), (0.75, True), (0.9, False), (0.6, True)])
def test_search_by_bow_kf_frame(gpu_vocab, frames, nnratio, check_ori):
    import slamhot
    m = slamhot.ORBmatcher(nnratio, check_ori)
    rng = np.random.default_rng(0)
    for j in range(1, len(frames)):
        k0, d0 = frames[0]
        k1, d1 = frames[j]
        valid = (rng.random(len(k0)) < 0.85).astype(np.uint8)
        A = _side(gpu_vocab, k0, d0, valid)
        B = _side(gpu_vocab, k1, d1, None)
        ng, b2a_g = m.SearchByBoW_KF_F(A, B)
        no, a2b_o, b2a_o = ob.search_by_bow(A, B, nnratio, check_ori, False)
        assert ng == no
        assert np.array_equal(b2a_g, b2a_o)
    m.close()


def test_search_by_bow_kf_kf(gpu_vocab, frames):
    import slamhot
    m = slamhot.ORBmatcher(0.75, True)
    rng = np.random.default_rng(1)
    k0, d0 = frames[0]
    for j in range(1, len(frames)):
        k1, d1 = frames[j]
        A = _side(gpu_vocab, k0, d0, (rng.random(len(k0)) < 0.9).astype(np.uint8))
        B = _side(gpu_vocab, k1, d1, (rng.random(len(k1)) < 0.9).astype(np.uint8))
        ng, a2b_g = m.SearchByBoW_KF_KF(A, B)
        no, a2b_o, b2a_o = ob.search_by_bow(A, B, 0.75, True, True)
        assert ng == no
        assert np.array_equal(a2b_g, a2b_o)
    m.close()


def test_search_by_bow_duplicates_and_ties(gpu_vocab):
    """Identical descriptors inside one node: ties must resolve to the first candidate."""
    import slamhot
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    d0 = np.repeat(base, 3, axis=0)
    d1 = np.repeat(base, 2, axis=0)
    k0 = np.zeros(len(d0), ob.KP_DTYPE)
    k1 = np.zeros(len(d1), ob.KP_DTYPE)
    k0["angle"] = rng.uniform(0, 360, len(d0)).astype(np.float32)
    k1["angle"] = rng.uniform(0, 360, len(d1)).astype(np.float32)
    m = slamhot.ORBmatcher(1.0, True)
    A = _side(gpu_vocab, k0, d0, None)
    B = _side(gpu_vocab, k1, d1, None)
    ng, b2a_g = m.SearchByBoW_KF_F(A, B)
    no, _, b2a_o = ob.search_by_bow(A, B, 1.0, True, False)
    assert ng == no and np.array_equal(b2a_g, b2a_o)
    m.close()


def test_bow_match_batch_device(gpu_vocab, vocab_arrays):
    """Device-resident extract -> ComputeBoW -> SearchByBoW over frame pairs equals the
    host path (oracle transform, FeatureVector, oracle SearchByBoW) on the same keypoints."""
    import torch

    import slamhot
    par, leaf, dn, wn = vocab_arrays
    img0 = synth.frame(11, 640, 480)
    imgs = np.stack([img0] + [synth.shifted(img0, dx, dy, a, 30 + i)
                              for i, (dx, dy, a) in enumerate([(3, 2, 2.0), (-5, 4, -6.0), (7, -2, 11.0)])])
    F, H, W = imgs.shape
    dev = torch.device("cuda", 0)
    ex = slamhot.ORBextractor(nfeatures=1000, max_size=(W, H), max_batch=F)
    cap = ex.cap
    d_img = torch.from_numpy(imgs).to(dev)
    d_kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(F, dtype=torch.int32, device=dev)
    d_mono = torch.zeros(F, dtype=torch.int32, device=dev)
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (3, 1)]
    d_a2b = torch.zeros((len(pairs), cap), dtype=torch.int32, device=dev)
    d_b2a = torch.zeros((len(pairs), cap), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(len(pairs), dtype=torch.int32, device=dev)
    rng = np.random.default_rng(3)
    valid = (rng.random((F, cap)) < 0.9).astype(np.uint8)
    d_valid = torch.from_numpy(valid).to(dev)
    m = slamhot.ORBmatcher(0.75, True)
    torch.cuda.synchronize()
    ex.extract_batch_device(d_img.data_ptr(), F, W, H, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(),
                            d_mono.data_ptr())
    torch.cuda.synchronize()
    m.bow_match_batch_device(gpu_vocab, F, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(), pairs,
                             d_a2b.data_ptr(), d_b2a.data_ptr(), d_nm.data_ptr(), d_valid=d_valid.data_ptr())
    assert m.bow_match_batch_status() == 0
    n = d_n.cpu().numpy()
    kps = d_kps.cpu().numpy().view(ob.KP_DTYPE)
    desc = d_desc.cpu().numpy()
    a2b, b2a, nm = d_a2b.cpu().numpy(), d_b2a.cpu().numpy(), d_nm.cpu().numpy()
    total = 0
    for p, (a, b) in enumerate(pairs):
        ka, da = kps[a, : n[a]].ravel(), desc[a, : n[a]]
        kb, db = kps[b, : n[b]].ravel(), desc[b, : n[b]]
        _, wta, nia = ob.vocab_transform(par, leaf, dn, wn, 6, da, 4)
        _, wtb, nib = ob.vocab_transform(par, leaf, dn, wn, 6, db, 4)
        A = (da, ka["angle"], valid[a, : n[a]]) + synth.feature_vector(nia, wta)
        B = (db, kb["angle"], None) + synth.feature_vector(nib, wtb)
        no, a2b_o, b2a_o = ob.search_by_bow(A, B, 0.75, True, False)
        assert nm[p] == no
        assert np.array_equal(a2b[p, : n[a]], a2b_o)
        assert np.array_equal(b2a[p, : n[b]], b2a_o)
        total += no
    assert total > 100
    # the same list again (its upload is skipped: same stream, same contents), then the reversed
    # list (uploaded): each pair's results follow it
    for plist in (pairs, pairs[::-1]):
        d_a2b.fill_(0)
        d_b2a.fill_(0)
        d_nm.fill_(0)
        torch.cuda.synchronize()
        m.bow_match_batch_device(gpu_vocab, F, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(), plist,
                                 d_a2b.data_ptr(), d_b2a.data_ptr(), d_nm.data_ptr(), d_valid=d_valid.data_ptr())
        assert m.bow_match_batch_status() == 0
        order = [pairs.index(pp) for pp in plist]
        assert np.array_equal(d_nm.cpu().numpy(), nm[order])
        assert np.array_equal(d_a2b.cpu().numpy(), a2b[order])
        assert np.array_equal(d_b2a.cpu().numpy(), b2a[order])
    m.close()
    ex.close()


def test_bow_match_batch_empty_frames(gpu_vocab, vocab_arrays):
    """Batched ComputeBoW + SearchByBoW with frames that have no keypoints (a flat image): pairs
    with an empty side match nothing (a2b / b2a all -1, count 0) and do not disturb the other
    pairs of the launch, which still equal the oracle."""
    import torch

    import slamhot
    par, leaf, dn, wn = vocab_arrays
    img0 = synth.frame(21, 640, 480)
    imgs = np.stack([img0, np.full((480, 640), 90, np.uint8), synth.shifted(img0, 4, -3, 5.0, 40)])
    F, H, W = imgs.shape
    dev = torch.device("cuda", 0)
    ex = slamhot.ORBextractor(nfeatures=1000, max_size=(W, H), max_batch=F)
    cap = ex.cap
    d_img = torch.from_numpy(imgs).to(dev)
    d_kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(F, dtype=torch.int32, device=dev)
    d_mono = torch.zeros(F, dtype=torch.int32, device=dev)
    pairs = [(0, 1), (1, 0), (1, 1), (0, 2), (2, 0)]
    d_a2b = torch.full((len(pairs), cap), 7, dtype=torch.int32, device=dev)
    d_b2a = torch.full((len(pairs), cap), 7, dtype=torch.int32, device=dev)
    d_nm = torch.full((len(pairs),), 7, dtype=torch.int32, device=dev)
    m = slamhot.ORBmatcher(0.75, True)
    torch.cuda.synchronize()
    ex.extract_batch_device(d_img.data_ptr(), F, W, H, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(),
                            d_mono.data_ptr())
    torch.cuda.synchronize()
    m.bow_match_batch_device(gpu_vocab, F, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(), pairs,
                             d_a2b.data_ptr(), d_b2a.data_ptr(), d_nm.data_ptr())
    assert m.bow_match_batch_status() == 0
    n = d_n.cpu().numpy()
    assert n[1] == 0 and n[0] > 500 and n[2] > 500
    kps = d_kps.cpu().numpy().view(ob.KP_DTYPE)
    desc = d_desc.cpu().numpy()
    a2b, b2a, nm = d_a2b.cpu().numpy(), d_b2a.cpu().numpy(), d_nm.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        if n[a] == 0 or n[b] == 0:
            assert nm[p] == 0
            assert (a2b[p, : n[a]] == -1).all() and (b2a[p, : n[b]] == -1).all()
            continue
        ka, da = kps[a, : n[a]].ravel(), desc[a, : n[a]]
        kb, db = kps[b, : n[b]].ravel(), desc[b, : n[b]]
        _, wta, nia = ob.vocab_transform(par, leaf, dn, wn, 6, da, 4)
        _, wtb, nib = ob.vocab_transform(par, leaf, dn, wn, 6, db, 4)
        A = (da, ka["angle"], None) + synth.feature_vector(nia, wta)
        B = (db, kb["angle"], None) + synth.feature_vector(nib, wtb)
        no, a2b_o, b2a_o = ob.search_by_bow(A, B, 0.75, True, False)
        assert nm[p] == no and no > 50
        assert np.array_equal(a2b[p, : n[a]], a2b_o)
        assert np.array_equal(b2a[p, : n[b]], b2a_o)
    m.close()
    ex.close()


@pytest.mark.parametrize("nfeatures, lo", [(500, 300), (1500, 1025), (3000, 2049)])
def test_bow_match_batch_feature_counts(gpu_vocab, vocab_arrays, nfeatures, lo):
    """k_featvec's two sorts: keypoint counts padding to 512 / 2048 (registers and wave shuffles,
    LDS only for partner distances >= 128) and past 2048 (the LDS bitonic), then SearchByBoW,
    against the oracle's FeatureVector and SearchByBoW."""
    import torch

    import slamhot
    par, leaf, dn, wn = vocab_arrays
    img0 = synth.frame(31, 1024, 768)
    imgs = np.stack([img0, synth.shifted(img0, 5, -3, 4.0, 41)])
    F, H, W = imgs.shape
    dev = torch.device("cuda", 0)
    ex = slamhot.ORBextractor(nfeatures=nfeatures, max_size=(W, H), max_batch=F)
    cap = ex.cap
    d_img = torch.from_numpy(imgs).to(dev)
    d_kps = torch.zeros((F, cap, 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(F, dtype=torch.int32, device=dev)
    d_mono = torch.zeros(F, dtype=torch.int32, device=dev)
    pairs = [(0, 1), (1, 0)]
    d_a2b = torch.zeros((len(pairs), cap), dtype=torch.int32, device=dev)
    d_b2a = torch.zeros((len(pairs), cap), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(len(pairs), dtype=torch.int32, device=dev)
    m = slamhot.ORBmatcher(0.75, True)
    torch.cuda.synchronize()
    ex.extract_batch_device(d_img.data_ptr(), F, W, H, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(),
                            d_mono.data_ptr())
    torch.cuda.synchronize()
    m.bow_match_batch_device(gpu_vocab, F, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(), pairs,
                             d_a2b.data_ptr(), d_b2a.data_ptr(), d_nm.data_ptr())
    assert m.bow_match_batch_status() == 0
    n = d_n.cpu().numpy()
    assert n.min() >= lo, n
    kps = d_kps.cpu().numpy().view(ob.KP_DTYPE)
    desc = d_desc.cpu().numpy()
    a2b, b2a, nm = d_a2b.cpu().numpy(), d_b2a.cpu().numpy(), d_nm.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        ka, da = kps[a, : n[a]].ravel(), desc[a, : n[a]]
        kb, db = kps[b, : n[b]].ravel(), desc[b, : n[b]]
        _, wta, nia = ob.vocab_transform(par, leaf, dn, wn, 6, da, 4)
        _, wtb, nib = ob.vocab_transform(par, leaf, dn, wn, 6, db, 4)
        A = (da, ka["angle"], None) + synth.feature_vector(nia, wta)
        B = (db, kb["angle"], None) + synth.feature_vector(nib, wtb)
        no, a2b_o, b2a_o = ob.search_by_bow(A, B, 0.75, True, False)
        assert nm[p] == no and no > 50
        assert np.array_equal(a2b[p, : n[a]], a2b_o)
        assert np.array_equal(b2a[p, : n[b]], b2a_o)
    m.close()
    ex.close()


def _clustered_desc(rng, n, centres, flips=1):
    """n descriptors drawn around a few centres (a few random bit flips each): most land in one
    vocabulary node, so nodes far above k_bow_match's 256-candidate tile appear."""
    d = centres[rng.integers(0, len(centres), n)].copy()
    for i in range(n):
        for b in rng.integers(0, 256, flips):
            d[i, b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def _kps(rng, n):
    k = np.zeros(n, ob.KP_DTYPE)
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    return k


@pytest.mark.parametrize("ncentres", [6, 14, 30, 60])
def test_search_by_bow_node_size_classes(gpu_vocab, ncentres):
    """Clustered descriptors whose FeatureVector nodes hold ~15 to ~150 candidates: the lane-group
    forms of k_bow_match (nodes of <= 16 / 32 / 64 B candidates, four / two / one per wave) and its
    wave loop (65..256) on one pair, against the oracle, KF-Frame and strict KF-KF."""
    import slamhot
    rng = np.random.default_rng(50 + ncentres)
    centres = rng.integers(0, 256, (ncentres, 32), dtype=np.uint8)
    d0, d1 = _clustered_desc(rng, 1100, centres, 2), _clustered_desc(rng, 1000, centres, 2)
    k0, k1 = _kps(rng, len(d0)), _kps(rng, len(d1))
    valid = (rng.random(len(d0)) < 0.9).astype(np.uint8)
    A = _side(gpu_vocab, k0, d0, valid)
    B = _side(gpu_vocab, k1, d1, None)
    sizes = np.diff(B[4])
    assert sizes.max() <= 256  # the tiled kernel, not the general one
    m = slamhot.ORBmatcher(0.9, True)
    ng, b2a_g = m.SearchByBoW_KF_F(A, B)
    no, _, b2a_o = ob.search_by_bow(A, B, 0.9, True, False)
    assert ng == no and np.array_equal(b2a_g, b2a_o)
    ng, a2b_g = m.SearchByBoW_KF_KF(A, B)
    no, a2b_o, _ = ob.search_by_bow(A, B, 0.9, True, True)
    assert ng == no and np.array_equal(a2b_g, a2b_o)
    m.close()


@pytest.mark.parametrize("strict", [False, True])
def test_search_by_bow_general_path_big_nodes(gpu_vocab, strict):
    """A node of B over 4 x 64 candidates: the unbounded kernel gives the oracle's matches."""
    import slamhot
    rng = np.random.default_rng(40)
    centres = rng.integers(0, 256, (2, 32), dtype=np.uint8)
    d0, d1 = _clustered_desc(rng, 900, centres), _clustered_desc(rng, 800, centres)
    k0, k1 = _kps(rng, len(d0)), _kps(rng, len(d1))
    valid = (rng.random(len(d0)) < 0.9).astype(np.uint8)
    A = _side(gpu_vocab, k0, d0, valid)
    B = _side(gpu_vocab, k1, d1, None)
    assert np.diff(B[4]).max() > 256  # the general path is exercised
    m = slamhot.ORBmatcher(0.9, True)
    if strict:
        ng, a2b_g = m.SearchByBoW_KF_KF(A, B)
        no, a2b_o, _ = ob.search_by_bow(A, B, 0.9, True, True)
        assert np.array_equal(a2b_g, a2b_o)
    else:
        ng, b2a_g = m.SearchByBoW_KF_F(A, B)
        no, _, b2a_o = ob.search_by_bow(A, B, 0.9, True, False)
        assert np.array_equal(b2a_g, b2a_o)
    assert ng == no and no > 0
    m.close()


def test_search_by_bow_general_path_large_sides(gpu_vocab):
    """Sides over k_bow_match's 8192-feature LDS tile."""
    import slamhot
    rng = np.random.default_rng(41)
    base = rng.integers(0, 256, (9000, 32), dtype=np.uint8)
    d0 = base.copy()
    d1 = base[rng.permutation(len(base))[:8500]].copy()
    for d in (d0, d1):
        for i in range(len(d)):
            b = rng.integers(0, 256)
            d[i, b >> 3] ^= np.uint8(1 << (b & 7))
    k0, k1 = _kps(rng, len(d0)), _kps(rng, len(d1))
    A = _side(gpu_vocab, k0, d0, None)
    B = _side(gpu_vocab, k1, d1, None)
    m = slamhot.ORBmatcher(0.75, False)
    ng, b2a_g = m.SearchByBoW_KF_F(A, B)
    no, _, b2a_o = ob.search_by_bow(A, B, 0.75, False, False)
    assert ng == no and no > 1000
    assert np.array_equal(b2a_g, b2a_o)
    m.close()


def test_bow_match_batch_general_pairs(gpu_vocab, vocab_arrays):
    """Batched path: pairs whose frame has a node over 256 candidates take the unbounded
    kernel (reported by the status call) and every pair's outputs equal the oracle's."""
    import torch

    import slamhot
    par, leaf, dn, wn = vocab_arrays
    rng = np.random.default_rng(42)
    centres = rng.integers(0, 256, (2, 32), dtype=np.uint8)
    F, cap = 4, 1200
    ns = [1100, 1000, 1200, 900]
    kps = np.zeros((F, cap), ob.KP_DTYPE)
    desc = np.zeros((F, cap, 32), np.uint8)
    for f in range(F):
        n = ns[f]
        d = _clustered_desc(rng, n, centres) if f in (1, 3) else rng.integers(0, 256, (n, 32), dtype=np.uint8)
        if f == 2:  # near-copies of frame 1 so that its pairs match
            d = desc[1, :n].copy()
            d[:, 0] ^= np.uint8(1)
        desc[f, :n] = d
        kps[f, :n] = _kps(rng, n)
    dev = torch.device("cuda", 0)
    d_kps = torch.from_numpy(kps.view(np.uint8).reshape(F, cap, 28).copy()).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_n = torch.tensor(ns, dtype=torch.int32, device=dev)
    pairs = [(0, 1), (2, 1), (1, 3), (0, 2), (3, 3)]
    d_a2b = torch.zeros((len(pairs), cap), dtype=torch.int32, device=dev)
    d_b2a = torch.zeros((len(pairs), cap), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(len(pairs), dtype=torch.int32, device=dev)
    m = slamhot.ORBmatcher(0.9, True)
    m.bow_match_batch_device(gpu_vocab, F, d_kps.data_ptr(), d_desc.data_ptr(), cap, d_n.data_ptr(), pairs,
                             d_a2b.data_ptr(), d_b2a.data_ptr(), d_nm.data_ptr())
    n_general = m.bow_match_batch_status()
    a2b, b2a, nm = d_a2b.cpu().numpy(), d_b2a.cpu().numpy(), d_nm.cpu().numpy()
    expect_general = 0
    for p, (a, b) in enumerate(pairs):
        _, wta, nia = ob.vocab_transform(par, leaf, dn, wn, 6, desc[a, : ns[a]], 4)
        _, wtb, nib = ob.vocab_transform(par, leaf, dn, wn, 6, desc[b, : ns[b]], 4)
        A = (desc[a, : ns[a]], kps[a, : ns[a]]["angle"], None) + synth.feature_vector(nia, wta)
        B = (desc[b, : ns[b]], kps[b, : ns[b]]["angle"], None) + synth.feature_vector(nib, wtb)
        expect_general += int(np.diff(B[4]).max() > 256)
        no, a2b_o, b2a_o = ob.search_by_bow(A, B, 0.9, True, False)
        assert nm[p] == no
        assert np.array_equal(a2b[p, : ns[a]], a2b_o)
        assert np.array_equal(b2a[p, : ns[b]], b2a_o)
    assert n_general == expect_general and n_general >= 2
    m.close()


def _write_vocab_text(path, parent, is_leaf, desc, weight, k, L, header=None):
    """ORBvoc.txt layout (TemplatedVocabulary.h:1350-1436): "k L scoring weighting", then one line
    per node after the root: parent, isLeaf, the 32 descriptor bytes (FORB::toString), weight."""
    lines = [header or f"{k} {L} 0 0"]
    for i in range(1, len(parent)):
        lines.append(f"{int(parent[i])} {int(is_leaf[i])} " + " ".join(str(int(b)) for b in desc[i]) +
                     f" {float(weight[i])!r}")
    path.write_text("\n".join(lines) + "\n")  # ORBvoc.txt ends with a newline


def test_vocab_load_text_equals_tables(tmp_path):
    """slamhot_vocab_load_text on a synthetic vocabulary written in the ORBvoc.txt format gives the
    same tree as the tables it was written from: identical transform (word, weight, node) for
    extracted descriptors; a malformed header is rejected like the reference (k > 20)."""
    import slamhot
    par, leaf, dn, wn = synth.vocab(10, 4, 3)
    p = tmp_path / "voc.txt"
    _write_vocab_text(p, par, leaf, dn, wn, 10, 4)
    vt = slamhot.Vocabulary(path=str(p))
    va = slamhot.Vocabulary(par, leaf, dn, wn, k=10, L=4)
    assert (vt.k, vt.L, vt.n_nodes, vt.n_words) == (va.k, va.L, va.n_nodes, va.n_words)
    _, d, _ = ob.extract(synth.frame(77, 640, 480))
    for lv in (0, 2, 4):
        a = vt.transform(d, lv)
        b = va.transform(d, lv)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    # and both equal the oracle's transform of the same tree
    w, wt, nid = ob.vocab_transform(par, leaf, dn, wn, 4, d, 2)
    a = vt.transform(d, 2)
    assert np.array_equal(a[0], w) and np.array_equal(a[1], wt) and np.array_equal(a[2], nid)
    vt.close()
    va.close()
    bad = tmp_path / "bad.txt"
    _write_vocab_text(bad, par, leaf, dn, wn, 10, 4, header="21 4 0 0")
    with pytest.raises(slamhot.SlamError):
        slamhot.Vocabulary(path=str(bad))
