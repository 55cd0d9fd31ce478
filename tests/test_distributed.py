"""The N>1 path of bench.py on CPU: two gloo ranks shard frames and BA windows exactly as the
nccl ranks do on GPUs (slamhot/dist.py), run the CPU oracle on their shard, and combine with
the same collectives (max time, summed units, gathered digests).  The combined result must
equal a single-process run over all units."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_bind as ob
from slamhot import dist as sdist
from slamhot import synth

N_FRAMES, N_WIN = 5, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frame_digest(idx, flip=None):
    """(keypoints, combined unit hashes) of frames idx; flip = frame whose first descriptor
    bit is flipped (a one-bit parity break on one rank)."""
    hs, count = [], 0
    for i in idx:
        img = synth.frame(700 + i, 320, 240)
        kps, desc, _ = ob.extract(img)
        if i == flip:
            desc = desc.copy()
            desc[0, 0] ^= 1
        hs.append(sdist.unit_hash(i, kps, desc))
        count += len(kps)
    return count, sdist.combine(hs)


def _lba_digest(idx):
    hs, iters = [], 0
    for i in idx:
        w = synth.lba_window(900 + i, n_kf=8, n_pt=60, obs_per_pt=3)
        r = ob.lba_solve(w)
        hs.append(sdist.unit_hash(i, r["kf_Tcw"], r["pt_pos"], r["edge_outlier"]))
        iters += r["iterations"][0] + r["iterations"][1]
    return iters, sdist.combine(hs)


def _worker(rank, world, port, q):
    import time

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t0 = time.perf_counter()
    fidx = sdist.shard(N_FRAMES, rank, world)
    kcount, kdig = _frame_digest(fidx)
    widx = sdist.shard(N_WIN, rank, world)
    lit, ldig = _lba_digest(widx)
    elapsed = time.perf_counter() - t0
    el_max, units = sdist.reduce_run(dist, "cpu", elapsed, float(len(fidx)))
    _, wunits = sdist.reduce_run(dist, "cpu", elapsed, float(len(widx)))
    kg = sdist.gather_digests(dist, "cpu", world, kcount, kdig)
    lg = sdist.gather_digests(dist, "cpu", world, lit, ldig)
    # the same gather with one descriptor bit flipped in one frame of rank 1
    _, fdig = _frame_digest(fidx, flip=fidx[0] if rank == 1 else None)
    fg = sdist.gather_digests(dist, "cpu", world, kcount, fdig)
    # setup broadcast of the replicated vocabulary tables (bench.py match leg)
    voc = sdist.broadcast_arrays(dist, "cpu", synth.vocab(4, 3, 7) if rank == 0 else None)
    q.put((rank, elapsed, el_max, units, wunits, kg, lg, sdist.digest(*voc), [(a.dtype.str, a.shape) for a in voc], fg))
    dist.destroy_process_group()


def test_unit_hashes_do_not_cancel():
    """Repeated content (the headline batch repeats its unique frames) must not cancel: the old
    XOR fold gave 0 for any even repetition; position-mixed unit hashes do not."""
    d = np.random.default_rng(0).integers(0, 256, (100, 32), dtype=np.uint8)
    hs = [sdist.unit_hash(i, d) for i in range(8)]
    assert len(set(hs)) == 8 and sdist.combine(hs) != 0
    assert sdist.combine(hs) == sdist.combine(hs[::-1])  # order-independent across ranks
    d2 = d.copy()
    d2[5, 3] ^= 0x10
    assert sdist.unit_hash(3, d2) != hs[3]
    assert sdist.unit_hash(3, d) != sdist.unit_hash(4, d)


def test_shard_partitions_units():
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            parts = [sdist.shard(n, r, world) for r in range(world)]
            assert sorted(sum(parts, [])) == list(range(n))


def test_two_rank_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    elapsed = [o[1] for o in out]
    for o in out:
        assert o[2] == pytest.approx(max(elapsed))
        assert o[3] == N_FRAMES and o[4] == N_WIN
        assert o[5] == out[0][5] and o[6] == out[0][6]  # every rank sees the same gather
    kg, lg = out[0][5], out[0][6]
    kc, kd = _frame_digest(range(N_FRAMES))
    assert sum(c for c, _ in kg) == kc
    assert sdist.combine(d for _, d in kg) == kd != 0
    li, ld = _lba_digest(range(N_WIN))
    assert sum(c for c, _ in lg) == li
    assert sdist.combine(d for _, d in lg) == ld != 0
    # one flipped descriptor bit on one rank changes the gathered job digest
    assert sdist.combine(d for _, d in out[0][9]) != kd
    ref = synth.vocab(4, 3, 7)
    for o in out:  # rank 1 received exactly rank 0's tables
        assert o[7] == sdist.digest(*ref)
        assert o[8] == [(np.asarray(a).dtype.str, np.asarray(a).shape) for a in ref]


# ---- configs[4]: whole stereo sequences sharded across ranks (bench.py track leg)
N_SEQS, SEQ_FRAMES = 3, 3


def _identity_maps(w=752, h=480):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    return [(xx, yy), (xx, yy)]


def _sequence_digest(idx):
    """The oracle tracking chain (tests/track_oracle.py) over sequences `idx`: per frame the
    counts and the pose, folded into (frames, digest)."""
    import track_oracle as to
    P = to.params()
    voc = synth.vocab(4, 3, 7)
    maps = _identity_maps()
    recs, frames = [], 0
    for s in idx:
        L, R, _ = synth.stereo_sequence(401 + s, SEQ_FRAMES)
        st = to.SeqState()
        for f in range(SEQ_FRAMES):
            r = to.step(P, voc, maps, st, L[f], R[f])
            recs.append(sdist.unit_hash(1000 * s + f, np.array([r["n"], r["stereo"], r["nbow"], r["ninl1"],
                                                                 r["nlocal"], r["ninl2"], r["is_kf"], r["lost"]],
                                                                np.int32), r["Tcw"].astype(np.float32)))
            frames += 1
    return frames, sdist.combine(recs)


def _seq_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sidx = sdist.shard(N_SEQS, rank, world)
    frames, dig = _sequence_digest(sidx)
    _, units = sdist.reduce_run(dist, "cpu", 1.0, float(frames))
    g = sdist.gather_digests(dist, "cpu", world, frames, dig)
    q.put((rank, units, g))
    dist.destroy_process_group()


def test_two_rank_gloo_sequence_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seq_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for o in out:
        assert o[1] == N_SEQS * SEQ_FRAMES and o[2] == out[0][2]
    frames, dig = _sequence_digest(range(N_SEQS))
    g = out[0][2]
    assert sum(c for c, _ in g) == frames
    assert sdist.combine(d for _, d in g) == dig != 0
