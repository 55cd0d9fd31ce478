"""GPU parity of the per-sequence stereo tracking chain (slamhot_tracker_*, BASELINE.json
configs[4]) against the oracle chain (tests/track_oracle.py), teacher-forced: before every step
the device's reference KeyFrame, pose, motion model (velocity, Tlr, reference pose) and last frame
are read back and handed to the oracle, which then runs the same step on the same raw images.
Per step and sequence: feature / stereo / TrackWithMotionModel / SearchByBoW /
TrackReferenceKeyFrame / SearchLocalPoints / TrackLocalMap counts and the motion / keyframe / lost
decisions are equal; the match arrays are equal (mvuRight, SearchByProjection(F, LastFrame),
SearchByBoW, SearchLocalPoints and the final mvpMapPoints); the pose within 1e-5; a new
KeyFrame's MapPoint set is equal and its points agree within 1e-5 (they unproject through the
step's optimized pose, itself within 1e-5)."""
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
        # sequence 1 moves faster: KeyFrames are inserted along it (CreateNewKeyFrame after the
        # initial one), sequence 0 keeps its initial KeyFrame
        L, R, _ = synth.stereo_sequence(301 + s, NFRAMES, step_m=0.03 if s == 0 else 0.07)
        out.append(([synth.unrectify(im, *maps[0]) for im in L], [synth.unrectify(im, *maps[1]) for im in R]))
    return maps, out


def _state_from_device(kf, ms):
    st = to.SeqState()
    st.initialized = bool(kf["initialized"])
    st.Tcw = kf["Tcw"].copy()
    st.n_ref = kf["n_ref"]
    if st.initialized:
        k = to.KeyFrame(kf["kps"], kf["desc"], None)
        k.valid, k.pos, k.normal = kf["mp_valid"], kf["mp_pos"], kf["mp_normal"]
        k.mind, k.maxd, k.mdesc = kf["mp_min_dist"], kf["mp_max_dist"], kf["mp_desc"]
        st.kf = k
        st.has_vel = bool(ms["has_vel"])
        st.V, st.Tlr, st.Tref, st.nkf = ms["V"], ms["Tlr"], ms["Tref"], ms["nkf"]
        st.last_kps, st.last_mp = ms["last_kps"], ms["last_mp"]
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
    n_kf = n_motion = 0
    for f in range(NFRAMES):
        states = [_state_from_device(T.keyframe(s), T.state(s)) for s in range(NSEQ)]
        dl = torch.from_numpy(np.stack([data[s][0][f] for s in range(NSEQ)])).to(dev)
        dr = torch.from_numpy(np.stack([data[s][1][f] for s in range(NSEQ)])).to(dev)
        torch.cuda.synchronize(dev)
        T.step_device(dl.data_ptr(), dr.data_ptr())
        recs = T.records()
        for s in range(NSEQ):
            o = to.step(P, voc_arrays, maps, states[s], data[s][0][f], data[s][1][f])
            g = recs[s]
            got = (g["n"], g["n_stereo"], g["n_motion"], g["motion"], g["n_bow"], g["n_inl_ref"], g["n_local"],
                   g["n_inl"], g["is_keyframe"], g["lost"], g["status"])
            exp = (o["n"], o["stereo"], o["n_motion"], o["motion"], o["nbow"], o["ninl1"], o["nlocal"], o["ninl2"],
                   o["is_kf"], o["lost"], 0)
            assert got == exp, (f, s, got, exp)
            assert np.abs(g["Tcw"] - o["Tcw"]).max() <= 1e-5, (f, s)
            n_motion += g["motion"]
            fr = T.frame(s)
            assert np.array_equal(fr["uright"], o["uright"]), (f, s)
            if g["initialized"] and f > 0:
                assert np.array_equal(fr["motion_match"], o["motion_match"]), (f, s)
                if not g["motion"]:
                    assert np.array_equal(fr["bow_match"], o["bow_match"]), (f, s)
                assert np.array_equal(fr["local_match"], o["local_match"]), (f, s)
                assert np.array_equal(fr["mappoints"], o["mappoints"]), (f, s)
            if o["is_kf"]:
                n_kf += 1
                kd = T.keyframe(s)
                ko = states[s].kf
                assert np.array_equal(kd["kps"].view(np.uint8), ko.kps.view(np.uint8))
                assert np.array_equal(kd["mp_valid"], ko.valid), (f, s)
                v = ko.valid.astype(bool)
                assert np.array_equal(kd["mp_desc"][v], ko.mdesc[v])
                assert np.abs(kd["mp_pos"][v] - ko.pos[v]).max() <= 1e-5
                assert np.abs(kd["mp_normal"][v] - ko.normal[v]).max() <= 1e-5
                assert kd["n_ref"] == int(v.sum())
        if f > 0:
            assert all(not r["lost"] for r in recs), recs
    assert n_kf >= NSEQ + 1  # the initial KeyFrames and at least one inserted later
    assert n_motion >= NSEQ * (NFRAMES - 3)  # TrackWithMotionModel tracked the steady-state frames
    T.close()
    voc.close()


def test_tracker_candidate_overflow_voids_step(seqs, monkeypatch):
    """A SearchByProjection candidate overflow (forced with a tiny candidate capacity) voids that
    sequence's step on the device: status 1, reported lost, and its pose / KeyFrame / motion state
    stay as before the step; slamhot_tracker_records reports SLAM_ECAP."""
    import torch

    import slamhot
    maps, data = seqs
    P = to.params()
    voc = slamhot.Vocabulary(*synth.vocab(10, 6, 0), k=10, L=6)
    cam = (P["fx"], P["fy"], P["cx"], P["cy"], P["bf"])
    monkeypatch.setenv("SLAMHOT_TRACK_CAND_CAP", "16")
    T = slamhot.Tracker(voc, NSEQ, cam, maps=maps)
    dev = torch.device("cuda", 0)
    for f in range(3):
        before = [(T.keyframe(s), T.state(s)) for s in range(NSEQ)]
        dl = torch.from_numpy(np.stack([data[s][0][f] for s in range(NSEQ)])).to(dev)
        dr = torch.from_numpy(np.stack([data[s][1][f] for s in range(NSEQ)])).to(dev)
        torch.cuda.synchronize(dev)
        T.step_device(dl.data_ptr(), dr.data_ptr())
        st, recs = T.records_status()
        if f == 0:
            assert st == 0 and all(r["is_keyframe"] for r in recs)  # StereoInitialization runs no search
            continue
        assert st == slamhot.SLAM_ECAP and all(r["status"] == 1 and r["lost"] for r in recs)
        for s in range(NSEQ):
            kb, sb = before[s]
            ka, sa = T.keyframe(s), T.state(s)
            assert np.array_equal(ka["Tcw"], kb["Tcw"]) and np.array_equal(ka["kps"].view(np.uint8), kb["kps"].view(np.uint8))
            assert np.array_equal(ka["mp_valid"], kb["mp_valid"]) and sa["has_vel"] == sb["has_vel"]
            assert np.array_equal(sa["last_mp"], sb["last_mp"]) and np.array_equal(sa["Tlr"], sb["Tlr"])
    T.close()
    voc.close()
