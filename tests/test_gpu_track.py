"""GPU parity of the per-sequence stereo tracking chain (slamhot_tracker_*, BASELINE.json
configs[4]) against the oracle chain (tests/track_oracle.py), teacher-forced: before every step
the device's reference KeyFrame and pose are read back and handed to the oracle, which then runs
the same step on the same raw images.  Per step and sequence: feature / stereo / SearchByBoW /
TrackReferenceKeyFrame / SearchLocalPoints / TrackLocalMap counts and the keyframe / lost
decisions are equal, the pose within 1e-5; a new KeyFrame's MapPoint set is equal and its points
agree within 1e-4 (they unproject through the step's optimized pose)."""
import numpy as np
import pytest

import track_oracle as to
from slamhot import synth

pytestmark = pytest.mark.gpu

NSEQ, NFRAMES = 2, 7


@pytest.fixture(scope="module")
def seqs():
    import bench
    maps = bench.euroc_maps()
    out = []
    for s in range(NSEQ):
        L, R, _ = synth.stereo_sequence(301 + s, NFRAMES)
        out.append(([synth.unrectify(im, *maps[0]) for im in L], [synth.unrectify(im, *maps[1]) for im in R]))
    return maps, out


def _state_from_device(kf):
    st = to.SeqState()
    st.initialized = bool(kf["initialized"])
    st.Tcw = kf["Tcw"].copy()
    st.n_ref = kf["n_ref"]
    if st.initialized:
        k = to.KeyFrame(kf["kps"], kf["desc"], None)
        k.valid, k.pos, k.normal = kf["mp_valid"], kf["mp_pos"], kf["mp_normal"]
        k.mind, k.maxd, k.mdesc = kf["mp_min_dist"], kf["mp_max_dist"], kf["mp_desc"]
        st.kf = k
    return st


def test_tracker_teacher_forced(seqs):
    import torch

    import slamhot
    maps, data = seqs
    P = to.params()
    voc_arrays = synth.vocab(10, 6, 0)
    voc = slamhot.Vocabulary(*voc_arrays, k=10, L=6)
    cam = (P["fx"], P["fy"], P["cx"], P["cy"], P["bf"])
    T = slamhot.Tracker(voc, NSEQ, cam, maps=maps)
    dev = torch.device("cuda", 0)
    n_kf = 0
    for f in range(NFRAMES):
        states = [_state_from_device(T.keyframe(s)) for s in range(NSEQ)]
        dl = torch.from_numpy(np.stack([data[s][0][f] for s in range(NSEQ)])).to(dev)
        dr = torch.from_numpy(np.stack([data[s][1][f] for s in range(NSEQ)])).to(dev)
        torch.cuda.synchronize(dev)
        T.step_device(dl.data_ptr(), dr.data_ptr())
        recs = T.records()
        for s in range(NSEQ):
            o = to.step(P, voc_arrays, maps, states[s], data[s][0][f], data[s][1][f])
            g = recs[s]
            got = (g["n"], g["n_stereo"], g["n_bow"], g["n_inl_ref"], g["n_local"], g["n_inl"], g["is_keyframe"], g["lost"])
            exp = (o["n"], o["stereo"], o["nbow"], o["ninl1"], o["nlocal"], o["ninl2"], o["is_kf"], o["lost"])
            assert got == exp, (f, s, got, exp)
            assert np.abs(g["Tcw"] - o["Tcw"]).max() <= 1e-5, (f, s)
            if o["is_kf"]:
                n_kf += 1
                kd = T.keyframe(s)
                ko = states[s].kf
                assert np.array_equal(kd["kps"].view(np.uint8), ko.kps.view(np.uint8))
                assert np.array_equal(kd["mp_valid"], ko.valid), (f, s)
                v = ko.valid.astype(bool)
                assert np.array_equal(kd["mp_desc"][v], ko.mdesc[v])
                assert np.abs(kd["mp_pos"][v] - ko.pos[v]).max() <= 1e-4
                assert np.abs(kd["mp_normal"][v] - ko.normal[v]).max() <= 1e-4
                assert kd["n_ref"] == int(v.sum())
        if f > 0:
            assert all(not r["lost"] for r in recs), recs
    assert n_kf >= NSEQ + 1  # the initial KeyFrames and at least one inserted later
    T.close()
    voc.close()
