"""numpy_twin — an independent numpy restatement of src/cpu.cc used to cross-check the C
oracle on small inputs.  TEST INFRASTRUCTURE ONLY.

Differs from the C oracle only where numpy forces it: sums use numpy's pairwise order and
the eigenvector comes from LAPACK (np.linalg.eigh) instead of Jacobi, so agreement is to
~1e-12, not bitwise — which is the point: two independent restatements of cpu.cc agree.
"""
from __future__ import annotations

import numpy as np


def closest(p: np.ndarray, m: np.ndarray):
    """cpu.cc:5-27 with ((dx^2 + dy^2) + dz^2) and first-min ties (np.argmin is first-min)."""
    d = p[:, None, :] - m[None, :, :]
    sq = d * d
    dist = (sq[..., 0] + sq[..., 1]) + sq[..., 2]
    idx = np.argmin(dist, axis=1).astype(np.int32)
    return m[idx], idx


def find_alignment(p: np.ndarray, y: np.ndarray):
    """cpu.cc:105-175 (Horn, quaternion from the largest eigenvalue)."""
    mu_p = p.mean(axis=0)
    mu_y = y.mean(axis=0)
    pp = p - mu_p
    yp = y - mu_y
    S = pp.T @ yp  # S(r, c) = sum p'_r y'_c  (cpu.cc:119)
    s = S
    N = np.array([
        [s[0, 0] + s[1, 1] + s[2, 2], s[1, 2] - s[2, 1], -s[0, 2] + s[2, 0], s[0, 1] - s[1, 0]],
        [-s[2, 1] + s[1, 2], s[0, 0] - s[2, 2] - s[1, 1], s[0, 1] + s[1, 0], s[0, 2] + s[2, 0]],
        [s[2, 0] - s[0, 2], s[1, 0] + s[0, 1], s[1, 1] - s[2, 2] - s[0, 0], s[1, 2] + s[2, 1]],
        [-s[1, 0] + s[0, 1], s[2, 0] + s[0, 2], s[2, 1] + s[1, 2], s[2, 2] - s[1, 1] - s[0, 0]],
    ])
    w, V = np.linalg.eigh(N)
    q0, q1, q2, q3 = V[:, int(np.argmax(w))]
    qbar = np.array([[q0, -q1, -q2, -q3], [q1, q0, q3, -q2], [q2, -q3, q0, q1], [q3, q2, -q1, q0]])
    qcap = np.array([[q0, -q1, -q2, -q3], [q1, q0, -q3, q2], [q2, q3, q0, -q1], [q3, -q2, q1, q0]])
    R = (qbar.T @ qcap)[1:, 1:]
    sc = np.sqrt((yp * yp).sum() / (pp * pp).sum())
    t = mu_y - sc * R @ mu_p
    q = p @ (sc * R).T + t
    err = float(((y - q) ** 2).sum())
    return sc, R, t, err


def icp(m: np.ndarray, p: np.ndarray, max_iter: int, threshold: float = 1e-5):
    """cpu.cc:55-79."""
    new_p = p.copy()
    errs = []
    for _ in range(max_iter):
        Y, _ = closest(new_p, m)
        s, R, t, e = find_alignment(new_p, Y)
        new_p = new_p @ (s * R).T + t
        e2 = float(((Y - new_p) ** 2).sum())
        err = (e + e2) / p.shape[0]
        errs.append(err)
        if err < threshold:
            break
    return new_p, np.array(errs)
