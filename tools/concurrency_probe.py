"""Probe: ORB extraction throughput with K extractor handles on K streams (B/K frames each)
vs one handle with B frames.  Prints frames/s per configuration."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam3-noted_amd")]
import torch  # noqa: E402

torch.cuda.init()
import slamhot  # noqa: E402
from slamhot import synth  # noqa: E402

W, H, B = 640, 480, 256
dev = torch.device("cuda", 0)
frames = synth.frames(range(64), W, H)
imgs = torch.from_numpy(np.concatenate([frames] * (B // 64))).to(dev)
for K in [int(k) for k in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2", "4"])]:
    nb = B // K
    exs = [slamhot.ORBextractor(nfeatures=1000, max_size=(W, H), max_batch=nb) for _ in range(K)]
    cap = exs[0].cap
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    outs = [(torch.zeros((nb, cap, 28), dtype=torch.uint8, device=dev), torch.zeros((nb, cap, 32), dtype=torch.uint8, device=dev),
             torch.zeros(nb, dtype=torch.int32, device=dev), torch.zeros(nb, dtype=torch.int32, device=dev)) for _ in range(K)]

    def step():
        for k in range(K):
            k_, d_, n_, m_ = outs[k]
            exs[k].extract_batch_device(imgs[k * nb:(k + 1) * nb].data_ptr(), nb, W, H, k_.data_ptr(), d_.data_ptr(),
                                        cap, n_.data_ptr(), m_.data_ptr(), stream=streams[k].cuda_stream)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 30
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"K={K}: {B * steps / dt:.0f} frames/s ({dt / steps * 1e3:.3f} ms/step)", flush=True)
    for e in exs:
        e.close()
