"""Multi-GPU plumbing of the batched path: one process per GPU, independent
units (frames, BA windows) sharded by rank, no collective on the data path.  The only
collectives are the timing reduction (max over ranks), the unit count (sum) and an all-gather
of per-rank parity digests at the end (each the sum of position-mixed unit hashes), plus one setup broadcast of the replicated tables (the
vocabulary) from rank 0.  Backend-agnostic: "nccl" (RCCL over xGMI) with
device tensors in bench.py, "gloo" with CPU tensors in the tests."""
from __future__ import annotations

import hashlib

import numpy as np


def shard(n_units: int, rank: int, world: int) -> list[int]:
    """Units owned by `rank`: i = rank (mod world)."""
    return list(range(rank, n_units, world))


MASK62 = (1 << 62) - 1


def _update(h, arrays):
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(f"{a.dtype.str}{a.shape}".encode())
        h.update(a.view(np.uint8).tobytes())


def digest(*arrays) -> int:
    """62-bit content hash (BLAKE2b) of byte arrays, dtype and shape included (fits int64)."""
    h = hashlib.blake2b(digest_size=8)
    _update(h, arrays)
    return int.from_bytes(h.digest(), "little") & MASK62


def unit_hash(index: int, *arrays) -> int:
    """Hash of one unit of work (a frame, a BA window, a sequence) mixed with its GLOBAL index, so
    equal outputs of different units never cancel and a unit computed on the wrong rank or in
    the wrong slot changes the result."""
    h = hashlib.blake2b(digest_size=8)
    h.update(int(index).to_bytes(8, "little", signed=True))
    _update(h, arrays)
    return int.from_bytes(h.digest(), "little") & MASK62


def combine(hashes) -> int:
    """Order-independent combination of unit hashes (sum mod 2^62): a rank combines its units,
    the gathered rank values combine the same way into the job's digest, which therefore equals
    a single-process run over all units whatever the sharding."""
    acc = 0
    for x in hashes:
        acc = (acc + int(x)) & MASK62
    return acc


def _coll_device(dist, device):
    """Collectives run on `device` under nccl, on the host under gloo (bench rehearsals)."""
    try:
        return "cpu" if dist.get_backend() == "gloo" else device
    except Exception:
        return device


def reduce_run(dist, device, elapsed_s: float, units: float):
    """(max elapsed over ranks, total units over ranks)."""
    import torch
    if dist is None:
        return elapsed_s, units
    device = _coll_device(dist, device)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    u = torch.tensor([units], dtype=torch.float64, device=device)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), float(u.item())


def gather_digests(dist, device, world: int, count: int, dig: int):
    """[(count, digest)] of every rank, in rank order."""
    import torch
    if dist is None:
        return [(count, dig)]
    device = _coll_device(dist, device)
    g = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(g, torch.tensor([count, dig], dtype=torch.int64, device=device))
    return [(int(x[0].item()), int(x[1].item())) for x in g]


def broadcast_arrays(dist, device, arrays):
    """Rank 0's numpy arrays on every rank (setup only: the vocabulary tree is built or loaded
    once and replicated).  `arrays` is ignored on ranks > 0.  Shapes and dtypes
    travel first (one int64 header), then one byte buffer."""
    import torch
    if dist is None:
        return [np.asarray(a) for a in arrays]
    device = _coll_device(dist, device)
    rank = dist.get_rank()
    codes = ["u1", "i1", "u2", "i2", "u4", "i4", "u8", "i8", "f4", "f8", "b1"]
    if rank == 0:
        arrs = [np.ascontiguousarray(a) for a in arrays]
        meta = [len(arrs)]
        for a in arrs:
            meta += [codes.index(a.dtype.str[1:]), a.ndim] + list(a.shape)
        hdr = torch.tensor([len(meta)] + meta + [0] * (255 - len(meta)), dtype=torch.int64, device=device)
    else:
        hdr = torch.zeros(256, dtype=torch.int64, device=device)
    dist.broadcast(hdr, src=0)
    h = hdr.cpu().numpy()
    meta = list(h[1:1 + int(h[0])])
    n, pos, specs = int(meta[0]), 1, []
    for _ in range(n):
        dt, nd = np.dtype(codes[int(meta[pos])]), int(meta[pos + 1])
        shape = tuple(int(v) for v in meta[pos + 2:pos + 2 + nd])
        specs.append((dt, shape))
        pos += 2 + nd
    sizes = [int(np.prod(sh)) * dt.itemsize for dt, sh in specs]
    total = sum(sizes)
    if rank == 0:
        buf = torch.from_numpy(np.concatenate([a.view(np.uint8).ravel() for a in arrs]) if total else
                               np.zeros(0, np.uint8)).to(device)
    else:
        buf = torch.zeros(total, dtype=torch.uint8, device=device)
    if total:
        dist.broadcast(buf, src=0)
    raw = buf.cpu().numpy()
    out, off = [], 0
    for (dt, sh), nb in zip(specs, sizes):
        out.append(raw[off:off + nb].view(dt).reshape(sh).copy())
        off += nb
    return out
