"""Multi-GPU plumbing of the batched path: one process per GPU, independent
units (frames, BA windows) sharded by rank, no collective on the data path.  The only
collectives are the timing reduction (max over ranks), the unit count (sum) and an all-gather
of per-rank parity digests at the end.  Backend-agnostic: "nccl" (RCCL over xGMI) with
device tensors in bench.py, "gloo" with CPU tensors in the tests."""
from __future__ import annotations

import numpy as np


def shard(n_units: int, rank: int, world: int) -> list[int]:
    """Units owned by `rank`: i = rank (mod world)."""
    return list(range(rank, n_units, world))


def digest(*arrays) -> int:
    """64-bit XOR-fold of byte arrays (order-independent across ranks, 62-bit so it fits int64)."""
    acc = np.uint64(0)
    for a in arrays:
        b = np.ascontiguousarray(a).view(np.uint8).ravel()
        pad = (-len(b)) % 8
        if pad:
            b = np.concatenate([b, np.zeros(pad, np.uint8)])
        if len(b):
            acc ^= np.bitwise_xor.reduce(b.view(np.uint64))
    return int(acc & np.uint64((1 << 62) - 1))


def reduce_run(dist, device, elapsed_s: float, units: float):
    """(max elapsed over ranks, total units over ranks)."""
    import torch
    if dist is None:
        return elapsed_s, units
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
    g = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(g, torch.tensor([count, dig], dtype=torch.int64, device=device))
    return [(int(x[0].item()), int(x[1].item())) for x in g]
