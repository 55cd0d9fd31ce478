"""Debug helper (GPU): run the device tracker on the test sequences and print every record and
the motion-model state, next to the free-running oracle chain."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "orb-slam3-noted_amd")]
import numpy as np
import torch

import bench
import slamhot
import track_oracle as to
from slamhot import synth

NSEQ, NF = 2, 7
maps = bench.euroc_maps()
P = to.params()
va = synth.vocab(10, 6, 0)
voc = slamhot.Vocabulary(*va, k=10, L=6)
T = slamhot.Tracker(voc, NSEQ, (P["fx"], P["fy"], P["cx"], P["cy"], P["bf"]), maps=maps)
data = []
for s in range(NSEQ):
    L, R, _ = synth.stereo_sequence(301 + s, NF)
    data.append(([synth.unrectify(im, *maps[0]) for im in L], [synth.unrectify(im, *maps[1]) for im in R]))
dev = torch.device("cuda", 0)
sts = [to.SeqState() for _ in range(NSEQ)]
for f in range(NF):
    dl = torch.from_numpy(np.stack([data[s][0][f] for s in range(NSEQ)])).to(dev)
    dr = torch.from_numpy(np.stack([data[s][1][f] for s in range(NSEQ)])).to(dev)
    torch.cuda.synchronize(dev)
    T.step_device(dl.data_ptr(), dr.data_ptr())
    recs = T.records()
    for s in range(NSEQ):
        g = recs[s]
        ms = T.state(s)
        o = to.step(P, va, maps, sts[s], data[s][0][f], data[s][1][f])
        print(f, s, "dev", {k: g[k] for k in ("n_motion", "motion", "n_bow", "n_inl_ref", "n_local", "n_inl", "is_keyframe", "lost")},
              "vel", ms["has_vel"], "nkf", ms["nkf"], "last_n", len(ms["last_mp"]), (ms["last_mp"] >= 0).sum())
        print(f, s, "ora", {k: o[k] for k in ("n_motion", "motion", "nbow", "ninl1", "nlocal", "ninl2", "is_kf", "lost")},
              "vel", sts[s].has_vel, "nkf", sts[s].nkf, "dT", float(np.abs(g["Tcw"] - o["Tcw"]).max()))
T.close()
voc.close()
