"""CPU model: per-cell sorted lists against the row walk -- dependent load rounds per query and per task (the cell lists measured and not kept)."""
import sys, numpy as np
from scipy.spatial import cKDTree
import os; _H = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, os.path.join(_H, "..", "iterative-closest-point_amd")); sys.path.insert(0, _H)
import icp_amd
from walk_model import fit
n = 1 << 18
m, p = icp_amd.synthetic_pair(n, seed=42, angle_deg=5.0)
lo, hi = m.min(0), m.max(0); ext = hi - lo
h = np.cbrt(np.prod(ext) * 2.0 / n); g = np.minimum(np.floor(ext / h) + 1, 4096).astype(int); inv = 1.0 / h
cell = np.clip(((m - lo) * inv).astype(int), 0, g - 1)
cnt = np.zeros(g[::-1], dtype=np.int32); np.add.at(cnt, (cell[:, 2], cell[:, 1], cell[:, 0]), 1)
pre = np.concatenate([np.zeros((g[2] * g[1], 1), np.int64), np.cumsum(cnt.reshape(-1, g[0]), 1)], 1)
# per-cell sorted list of the 27-neighbourhood by distance to the cell box (cell units)
tm = (m - lo) * inv
order = np.lexsort((cell[:, 0], cell[:, 1], cell[:, 2]))
tm_s = tm[order]; cid_s = (cell[order, 2] * g[1] + cell[order, 1]) * g[0] + cell[order, 0]
cstart = np.searchsorted(cid_s, np.arange(g.prod() + 1))
tree = cKDTree(m)
d, idx = tree.query(p); q = p.copy()
def morton(t):
    v = np.clip((t / g * 256).astype(np.int64), 0, 255); k = np.zeros(len(t), np.int64)
    for b in range(8):
        for a in range(3): k |= ((v[:, a] >> b) & 1) << (3 * b + a)
    return k
for it in range(1, 30):
    s, R, t = fit(q, m[idx]); q = s * q @ R.T + t
    e = ((q - m[idx]) ** 2).sum(1); r = np.sqrt(e) * inv
    if it not in (1, 5, 15, 29):
        d, idx = tree.query(q); continue
    tq = (q - lo) * inv
    perm = np.argsort(morton(tq), kind="stable")
    tqs, rs = tq[perm], r[perm]
    qc = np.clip(tqs.astype(int), 0, g - 1)
    # list entries within r of the cell box, from the 27 neighbours
    nent = np.zeros(n); nlist = np.zeros(n)
    for oz in (-1, 0, 1):
        for oy in (-1, 0, 1):
            for ox in (-1, 0, 1):
                c = qc + np.array([ox, oy, oz])
                ok = ((c >= 0) & (c < g)).all(1)
                cc = np.where(ok[:, None], c, 0)
                ci = (cc[:, 2] * g[1] + cc[:, 1]) * g[0] + cc[:, 0]
                a, b = cstart[ci], cstart[ci + 1]
                nlist += np.where(ok, b - a, 0)
                mx = (b - a).max()
                for j in range(mx):
                    kk = np.minimum(a + j, n - 1); val = ok & (a + j < b)
                    pt = tm_s[kk]
                    dd = np.maximum(0, np.maximum(qc - pt, pt - (qc + 1)))
                    nent += val & ((dd ** 2).sum(1) <= rs ** 2)
    # current walk: rows dealt 2 a lane (4 a query a round), points 2 at a time
    c0 = np.clip(((tqs - rs[:, None])).astype(int), 0, g - 1); c1 = np.clip(((tqs + rs[:, None])).astype(int), 0, g - 1)
    span = c1 - c0 + 1; nrq = span[:, 1] * span[:, 2]
    steps_walk = np.zeros(n)  # per query: max over its two lanes of dependent load steps
    lane_steps = np.zeros((n, 2))
    for r0 in range(0, nrq.max(), 4):
        for lanei in range(2):
            pts = np.zeros(n)
            any_row = np.zeros(n, bool)
            for v in range(2):
                rr = r0 + lanei + 2 * v
                okr = rr < nrq
                ry = rr % np.maximum(span[:, 1], 1); rz = rr // np.maximum(span[:, 1], 1)
                gy = np.minimum(c0[:, 1] + ry, g[1] - 1); gz = np.minimum(c0[:, 2] + rz, g[2] - 1)
                rowi = gz * g[1] + gy
                pts += np.where(okr, pre[rowi, c1[:, 0] + 1] - pre[rowi, c0[:, 0]], 0)
                any_row |= okr
            lane_steps[:, lanei] += np.where(any_row, 1 + np.ceil(pts / 2), 0)
    steps_walk = lane_steps.max(1)
    steps_list = np.ceil(np.maximum(nent, 1) / 8)
    T = n // 32
    wmax = lambda x: x.reshape(T, 32).max(1).mean()
    print(f"it {it}: r {rs.mean():.3f} cells | list scanned {nent.mean():.2f} (27-nbhd {nlist.mean():.1f}), fallback r>=1: {(rs >= 0.999).mean()*100:.3f}% "
          f"| dependent steps/query walk {steps_walk.mean():.2f} (wave max {wmax(steps_walk):.2f}) list {steps_list.mean():.2f} (wave max {wmax(steps_list):.2f})")
    d, idx = tree.query(q)
