"""Seeded synthetic inputs of the shapes BASELINE.json names (no datasets in this image).

Frames: procedural u8 textures (random rectangles + Gaussian blobs + value noise, clipped to
[0, 255]) as SURVEY.md §8(d) config 2 specifies.  Everything is derived from
``numpy.random.default_rng(seed)`` so a seed fully determines a frame.
"""
from __future__ import annotations

import numpy as np


def _value_noise(rng: np.random.Generator, h: int, w: int, cell: int) -> np.ndarray:
    gh, gw = h // cell + 2, w // cell + 2
    grid = rng.random((gh, gw), dtype=np.float64)
    ys = np.arange(h) / cell
    xs = np.arange(w) / cell
    y0 = ys.astype(np.int64)
    x0 = xs.astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    fy = fy * fy * (3 - 2 * fy)
    fx = fx * fx * (3 - 2 * fx)
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    return (g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy


def frame(seed: int, width: int = 640, height: int = 480) -> np.ndarray:
    """One textured grayscale frame (height, width) uint8."""
    rng = np.random.default_rng(seed)
    img = 90.0 + 60.0 * _value_noise(rng, height, width, 48)
    img += 25.0 * _value_noise(rng, height, width, 9)
    for _ in range(60):
        x0, y0 = rng.integers(0, width), rng.integers(0, height)
        rw, rh = rng.integers(8, 120), rng.integers(8, 120)
        img[y0:y0 + rh, x0:x0 + rw] += rng.uniform(-70, 70)
    for _ in range(25):
        cx, cy = rng.uniform(0, width), rng.uniform(0, height)
        s = rng.uniform(3, 25)
        amp = rng.uniform(-80, 80)
        r = int(np.ceil(4 * s))
        x0, x1 = max(0, int(cx) - r), min(width, int(cx) + r + 1)
        y0, y1 = max(0, int(cy) - r), min(height, int(cy) + r + 1)
        if x0 >= x1 or y0 >= y1:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1]
        img[y0:y1, x0:x1] += amp * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))
    img += rng.normal(0.0, 4.0, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def frames(seeds, width: int = 640, height: int = 480) -> np.ndarray:
    """Stack of frames (n, height, width) uint8."""
    return np.stack([frame(int(s), width, height) for s in seeds])


def shifted(img: np.ndarray, dx: float, dy: float, angle_deg: float, seed: int) -> np.ndarray:
    """Rigidly warped copy (nearest neighbour) plus light noise: a 'next frame' for matching."""
    h, w = img.shape
    rng = np.random.default_rng(seed)
    a = np.deg2rad(angle_deg)
    ca, sa = np.cos(a), np.sin(a)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    cx, cy = w / 2, h / 2
    xs = ca * (xx - cx - dx) + sa * (yy - cy - dy) + cx
    ys = -sa * (xx - cx - dx) + ca * (yy - cy - dy) + cy
    xi = np.clip(np.rint(xs), 0, w - 1).astype(np.int64)
    yi = np.clip(np.rint(ys), 0, h - 1).astype(np.int64)
    out = img[yi, xi].astype(np.float64) + rng.normal(0.0, 2.0, size=img.shape)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def vocab(k: int = 10, L: int = 6, seed: int = 0, stop_frac: float = 0.01):
    """Synthetic DBoW2-shaped vocabulary in breadth-first node order (node 0 = root):
    returns (parent int32, is_leaf uint8, desc (n,32) uint8, weight float64).  Node
    descriptors are random; a child is its parent with ~25% of bits flipped, so nearby
    descriptors descend alike.  A fraction of words get weight 0 (stopped words)."""
    rng = np.random.default_rng(seed)
    n = (k ** (L + 1) - 1) // (k - 1)
    parent = np.empty(n, np.int32)
    parent[0] = -1
    idx = np.arange(1, n)
    parent[1:] = (idx - 1) // k
    desc = np.empty((n, 32), np.uint8)
    desc[0] = rng.integers(0, 256, 32, dtype=np.uint8)
    first = 1
    for lvl in range(1, L + 1):
        cnt = k ** lvl
        par = desc[parent[first:first + cnt]]
        flips = rng.random((cnt, 256)) < 0.25
        bits = np.unpackbits(par, axis=1, bitorder="little") ^ flips.astype(np.uint8)
        desc[first:first + cnt] = np.packbits(bits, axis=1, bitorder="little")
        first += cnt
    is_leaf = np.zeros(n, np.uint8)
    nleaf = k ** L
    is_leaf[n - nleaf:] = 1
    weight = np.zeros(n, np.float64)
    w = rng.uniform(0.5, 3.0, nleaf)
    w[rng.random(nleaf) < stop_frac] = 0.0
    weight[n - nleaf:] = w
    return parent, is_leaf, desc, weight


def feature_vector(node_id: np.ndarray, weight: np.ndarray):
    """DBoW2 FeatureVector as CSR from per-feature (node id, word weight): features whose
    word weight is <= 0 are dropped (TemplatedVocabulary.h:1169), ascending node ids,
    ascending feature indices (FeatureVector::addFeature, FeatureVector.cpp:31-45)."""
    keep = np.nonzero(weight > 0)[0]
    nid = node_id[keep]
    order = np.lexsort((keep, nid))
    nid_s = nid[order]
    feats = keep[order].astype(np.uint32)
    uniq, starts = np.unique(nid_s, return_index=True)
    off = np.append(starts, len(nid_s)).astype(np.int32)
    return uniq.astype(np.uint32), off, feats
