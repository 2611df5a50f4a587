"""CPU model of the seeded grid search's work per query at C4 (nn_grid_resolve_kernel, all-mode):
cells, x-runs (rows) and model points each query's complete box covers, for cell sizes around
the grid's (2 points per cell) and with the rows clipped to the seed sphere (rows whose (y, z)
gap to the query exceeds the seed distance are skipped, the others narrowed in x to the chord).

    python tools/box_model.py [--queries 100000] [--residual-deg 0.3]

The scene is the model under a small residual rigid motion (an iteration near convergence) and
each query's seed is its nearest model point under a slightly larger residual (the previous
iteration's correspondence), as in icp_run's seeded iterations.
"""
import argparse

import numpy as np
from scipy.spatial import cKDTree


def rot(deg, axis=(1.0, 2.0, 3.0)):
    a = np.asarray(axis) / np.linalg.norm(axis)
    t = np.deg2rad(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", type=int, default=1 << 20)
    ap.add_argument("--queries", type=int, default=100000)
    ap.add_argument("--residual-deg", type=float, default=0.3)
    a = ap.parse_args()
    rng = np.random.default_rng(42)
    m = rng.uniform(-1, 1, size=(a.model, 3))
    sel = rng.choice(a.model, a.queries, replace=False)
    r, t = rot(a.residual_deg), np.array([0.004, -0.003, 0.002])
    q = m[sel] @ r.T + t
    q_prev = m[sel] @ rot(1.3 * a.residual_deg).T + 1.3 * t
    tree = cKDTree(m)
    _, seed = tree.query(q_prev)
    d2 = ((q - m[seed]) ** 2).sum(1)
    d_nn, _ = tree.query(q)
    print(f"seed R median {np.median(np.sqrt(d2)):.4f}  NN dist median {np.median(d_nn):.4f}")
    lo, hi = m.min(0), m.max(0)
    h0 = np.cbrt(np.prod(hi - lo) * 2.0 / a.model)
    for f in (0.63, 0.8, 1.0, 1.26, 1.59):
        h = h0 * f
        g = (np.floor((hi - lo) / h) + 1).astype(int)
        cell = np.clip(np.floor((m - lo) / h).astype(int), 0, g - 1)
        cnt = np.zeros(g, dtype=np.int64)
        np.add.at(cnt, (cell[:, 0], cell[:, 1], cell[:, 2]), 1)
        cx = np.concatenate([np.zeros((1, g[1], g[2]), np.int64), np.cumsum(cnt, 0)], 0)  # x prefix per row
        R = np.sqrt(d2)
        c0 = np.clip(np.floor((q - R[:, None] - lo) / h).astype(int), 0, g - 1)
        c1 = np.clip(np.floor((q + R[:, None] - lo) / h).astype(int), 0, g - 1)
        ext = c1 - c0 + 1
        cells = ext.prod(1)
        rows = ext[:, 1] * ext[:, 2]
        pts = np.zeros(len(q), np.int64)
        rows_c = np.zeros(len(q), np.int64)
        pts_c = np.zeros(len(q), np.int64)
        for dy in range(ext[:, 1].max()):
            for dz in range(ext[:, 2].max()):
                live = (dy < ext[:, 1]) & (dz < ext[:, 2])
                cy, cz = c0[:, 1] + dy, c0[:, 2] + dz
                cyc, czc = np.minimum(cy, g[1] - 1), np.minimum(cz, g[2] - 1)
                full = cx[c1[:, 0] + 1, cyc, czc] - cx[c0[:, 0], cyc, czc]
                pts += np.where(live, full, 0)
                gy = np.maximum(0, np.maximum(lo[1] + cy * h - q[:, 1], q[:, 1] - (lo[1] + (cy + 1) * h)))
                gz = np.maximum(0, np.maximum(lo[2] + cz * h - q[:, 2], q[:, 2] - (lo[2] + (cz + 1) * h)))
                rem = d2 - gy * gy - gz * gz
                keep = live & (rem >= 0)
                rx = np.sqrt(np.maximum(rem, 0))
                x0 = np.clip(np.floor((q[:, 0] - rx - lo[0]) / h).astype(int), 0, g[0] - 1)
                x1 = np.clip(np.floor((q[:, 0] + rx - lo[0]) / h).astype(int), 0, g[0] - 1)
                clip = cx[x1 + 1, cyc, czc] - cx[x0, cyc, czc]
                rows_c += keep
                pts_c += np.where(keep, clip, 0)
        print(f"h x{f:4.2f} ({8 * f ** 3 * 2 / 8:4.2f} pts/cell): cells {cells.mean():6.1f}  rows {rows.mean():5.2f} "
              f"pts {pts.mean():6.1f} | clipped rows {rows_c.mean():5.2f} pts {pts_c.mean():6.1f}  "
              f"(p99 pts {np.percentile(pts, 99):.0f} / {np.percentile(pts_c, 99):.0f})")


if __name__ == "__main__":
    main()
