"""CPU model: candidates (points at least as close as the seed) per query and per 32-query task over a C4 registration."""
import sys, numpy as np
from scipy.spatial import cKDTree
import os; _H = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, os.path.join(_H, "..", "iterative-closest-point_amd")); sys.path.insert(0, _H)
import icp_amd
from walk_model import fit
n = 1 << 18
m, p = icp_amd.synthetic_pair(n, seed=42, angle_deg=5.0)
lo = m.min(0); h = np.cbrt(np.prod(m.max(0) - lo) * 2.0 / n)
tree = cKDTree(m)
d, idx = tree.query(p); q = p.copy()
g = 64
v = np.clip(((p - lo) / (2.0 / 256)).astype(np.int64), 0, 255); key = np.zeros(n, np.int64)
for b in range(8):
    for a in range(3): key |= ((v[:, a] >> b) & 1) << (3 * b + a)
perm = np.argsort(key, kind="stable")
for it in range(1, 30):
    s, R, t = fit(q, m[idx]); qn = s * q @ R.T + t
    e = ((qn - m[idx]) ** 2).sum(1)
    cnt = np.array([len(x) for x in tree.query_ball_point(qn, np.sqrt(e) * (1 + 1e-9))]) - 1
    d, idxn = tree.query(qn)
    ch = idxn != idx
    wave_c = (cnt[perm].reshape(-1, 32) > 0).any(1).mean()
    wave_c2 = np.maximum.reduce(cnt[perm].reshape(-1, 32), axis=1).mean()
    move = np.sqrt(((qn - q) ** 2).sum(1)) / h
    if it in (1, 2, 3, 5, 8, 12, 20, 29):
        print(f"it {it:2d}: move {move.mean():.3f} cells, NN changed {ch.mean()*100:.1f}%, candidates/query {cnt.mean():.3f}, waves with a candidate {wave_c*100:.0f}%, wave max cand {wave_c2:.2f}")
    q, idx = qn, idxn
