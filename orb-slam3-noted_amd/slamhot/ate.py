"""Absolute trajectory error, as the reference's evaluation scripts compute it
(evaluation/evaluate_ate_scale.py + evaluation/associate.py): trajectory text files
("stamp tx ty tz qx qy qz qw", ',' or whitespace separated, '#' comments), greedy timestamp
association, Horn closed-form alignment with the SVD sign fix and the scale
s = sum(data^T R model) / sum(|model|^2), and the printed triple
"rmse_SE3, scale, rmse_Sim3" (evaluate_ate_scale.py:189).  numpy restatement (no np.matrix),
checked against golden vectors produced with the reference's own functions
(tools/make_ate_golden.py -> tests/golden/ate.npz)."""
from __future__ import annotations

import numpy as np


def read_file_list(filename: str, remove_bounds: bool = False) -> dict:
    """associate.py:49-71."""
    with open(filename) as f:
        data = f.read()
    lines = data.replace(",", " ").replace("\t", " ").split("\n")
    if remove_bounds:
        lines = lines[100:-100]
    rows = [[v.strip() for v in line.split(" ") if v.strip() != ""] for line in lines
            if len(line) > 0 and line[0] != "#"]
    return dict((float(r[0]), r[1:]) for r in rows if len(r) > 1)


def associate(first: dict, second: dict, offset: float, max_difference: float):
    """associate.py:73-106: every candidate pair with |a - (b + offset)| < max_difference,
    sorted by (difference, a, b), taken greedily; returns matches sorted by a."""
    a = np.array(sorted(first.keys()), dtype=np.float64)
    b = np.array(sorted(second.keys()), dtype=np.float64)
    cands = []
    if len(a) and len(b):
        bo = b + offset
        lo = np.searchsorted(bo, a - max_difference, side="left")
        hi = np.searchsorted(bo, a + max_difference, side="right")
        for i in range(len(a)):
            for j in range(lo[i], hi[i]):
                d = abs(a[i] - (b[j] + offset))
                if d < max_difference:
                    cands.append((d, a[i], b[j]))
    cands.sort()
    used_a, used_b, matches = set(), set(), []
    for d, x, y in cands:
        if x not in used_a and y not in used_b:
            used_a.add(x)
            used_b.add(y)
            matches.append((x, y))
    matches.sort()
    return matches


def align(model: np.ndarray, data: np.ndarray):
    """evaluate_ate_scale.py:49-99 (Horn closed form with scale).  model, data: 3 x n.
    Returns rot, transGT, trans_errorGT, trans, trans_error, s."""
    model = np.asarray(model, np.float64)
    data = np.asarray(data, np.float64)
    mm = model.mean(1, keepdims=True)
    dm = data.mean(1, keepdims=True)
    mz = model - mm
    dz = data - dm
    W = np.zeros((3, 3))
    for c in range(model.shape[1]):
        W += np.outer(mz[:, c], dz[:, c])
    U, _, Vh = np.linalg.svd(W.T)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vh) < 0:
        S[2, 2] = -1
    rot = U @ S @ Vh
    rotmodel = rot @ mz
    dots = 0.0
    norms = 0.0
    for c in range(dz.shape[1]):
        dots += float(dz[:, c] @ rotmodel[:, c])
        ni = np.linalg.norm(mz[:, c])
        norms += ni * ni
    s = float(dots / norms)
    transGT = dm - s * rot @ mm
    trans = dm - rot @ mm
    errGT = s * rot @ model + transGT - data
    err = rot @ model + trans - data
    trans_errorGT = np.sqrt(np.sum(errGT * errGT, 0))
    trans_error = np.sqrt(np.sum(err * err, 0))
    return rot, transGT, trans_errorGT, trans, trans_error, s


def evaluate(first: dict, second: dict, offset: float = 0.0, scale: float = 1.0,
             max_difference: float = 20000000):
    """evaluate_ate_scale.py:149-189 -> (rmse_SE3, s, rmse_Sim3, n_pairs)."""
    matches = associate(first, second, float(offset), float(max_difference))
    if len(matches) < 2:
        raise ValueError("Couldn't find matching timestamp pairs between groundtruth and estimated trajectory!")
    first_xyz = np.array([[float(v) for v in first[a][0:3]] for a, b in matches]).T
    second_xyz = np.array([[float(v) * float(scale) for v in second[b][0:3]] for a, b in matches]).T
    rot, transGT, errGT, trans, err, s = align(second_xyz, first_xyz)
    rmse = float(np.sqrt(np.dot(err, err) / len(err)))
    rmseGT = float(np.sqrt(np.dot(errGT, errGT) / len(errGT)))
    return rmse, s, rmseGT, len(matches)
