"""Debug: GPU stereo batch vs host oracle pipeline on the bench's seeds."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam3-noted_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

torch.cuda.init()
import oracle_bind as ob  # noqa: E402
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

MBF = synth.EUROC_STEREO["bf"]
MB = MBF / synth.EUROC_STEREO["fx"]
P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 500
prs = [synth.stereo_pair(seed0 + s, 752, 480) for s in range(P)]
il = np.stack([p[0] for p in prs])
ir = np.stack([p[1] for p in prs])
left = slamhot.ORBextractor(nfeatures=1200, max_size=(752, 480), max_batch=P)
right = slamhot.ORBextractor(nfeatures=1200, max_size=(752, 480), max_batch=P)
out = slamhot.ComputeStereoMatches(left, right, il, ir, MBF, MB)
p = ob.params(nfeatures=1200)
sc, isc, _, _, _ = ob.levels(p)
for f in (0, P - 1):
    kl, dl, kr, dr, ur, dep = out[f]
    hkl, hdl, _ = ob.extract(il[f], p)
    hkr, hdr, _ = ob.extract(ir[f], p)
    print("frame", f, "n", len(kl), len(kr), "host n", len(hkl), len(hkr),
          "kps eq", np.array_equal(kl.view(np.uint8), hkl.view(np.uint8)),
          np.array_equal(kr.view(np.uint8), hkr.view(np.uint8)))
    pl = [left.pyramid_level(l, f) for l in range(8)]
    pr = [right.pyramid_level(l, f) for l in range(8)]
    hpl, hpr = ob.pyramid(il[f], p), ob.pyramid(ir[f], p)
    print("  pyr eq", [np.array_equal(a, b) for a, b in zip(pl, hpl)], [np.array_equal(a, b) for a, b in zip(pr, hpr)])
    u1, _ = ob.stereo_matches(hkl, hdl, hkr, hdr, hpl, hpr, sc, isc, MBF, MB)
    print("  gpu matches", (ur >= 0).sum(), "host pipeline matches", (u1 >= 0).sum())

# the bench's mode: one user stream, no host sync between the three calls
dev = torch.device("cuda", 0)
cap = left.cap
d_il, d_ir = torch.from_numpy(il).to(dev), torch.from_numpy(ir).to(dev)
bufs = [(torch.zeros((P, cap, 28), dtype=torch.uint8, device=dev), torch.zeros((P, cap, 32), dtype=torch.uint8, device=dev),
         torch.zeros(P, dtype=torch.int32, device=dev), torch.zeros(P, dtype=torch.int32, device=dev)) for _ in range(2)]
d_ur = torch.empty((P, cap), dtype=torch.float32, device=dev)
d_dep = torch.empty((P, cap), dtype=torch.float32, device=dev)
stream = torch.cuda.Stream(dev)
sm = slamhot.StereoMatcher()
torch.cuda.synchronize()
for ex, img, (k, d, n, m) in ((left, d_il, bufs[0]), (right, d_ir, bufs[1])):
    ex.extract_batch_device(img.data_ptr(), P, 752, 480, k.data_ptr(), d.data_ptr(), cap, n.data_ptr(), m.data_ptr(),
                            stream=stream.cuda_stream)
if len(sys.argv) > 3:
    torch.cuda.synchronize()
(kl, dl, nl, _), (kr, dr, nr, _) = bufs
sm.match_batch_device(left, right, P, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(), kr.data_ptr(), dr.data_ptr(),
                      nr.data_ptr(), cap, MBF, MB, d_ur.data_ptr(), d_dep.data_ptr(), stream=stream.cuda_stream)
torch.cuda.synchronize()
nl_h = nl.cpu().numpy()
klh = kl.cpu().numpy().view(ob.KP_DTYPE)
ur = d_ur.cpu().numpy()
for f in (0, P - 1):
    print("stream mode frame", f, "n", nl_h[f], "kps eq", np.array_equal(klh[f, :nl_h[f]].ravel().view(np.uint8),
                                                                          out[f][0].view(np.uint8)),
          "matches", (ur[f, :nl_h[f]] >= 0).sum(), "prev", (out[f][4] >= 0).sum())
