"""CPU model (tools/cert_model.py) of the exclusion-radius certificate over a C4 registration.

Per query the fused grid iteration keeps R, a lower bound on the distance from its position to
every model point other than its correspondence.  A walk (the seeded search) sets R = min(d2,
sqrt(e) + skin) -- d2 the second-nearest distance, e the seed distance, skin the extra radius the
walk scans -- and each later iteration lowers R by the query's motion.  A query whose seed
distance is below R keeps its correspondence without a walk (the certificate).

The model counts, per iteration: the queries that walk, and the 32-query chunks (slot order = the
scene's Morton order) that hold at least one.  scipy's kd-tree stands in for the exact search; the
transform is a plain similarity fit (statistics only, not the engine's bits).

    python tools/cert_model.py [--n 1048576] [--iters 30]
"""
import argparse
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/iterative-closest-point_amd")
import icp_amd  # noqa: E402


def fit(p, y):
    cp, cy = p.mean(0), y.mean(0)
    P, Y = p - cp, y - cy
    U, S, Vt = np.linalg.svd(Y.T @ P)
    D = np.diag([1, 1, np.sign(np.linalg.det(U @ Vt))])
    R = U @ D @ Vt
    s = np.sqrt((Y * Y).sum() / (P * P).sum())
    return s, R, cy - s * R @ cp


def morton(x, lo, hi, bits=10):
    c = np.clip(((x - lo) / (hi - lo) * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    k = np.zeros(len(x), np.int64)
    for b in range(bits):
        for a in range(3):
            k |= ((c[:, a] >> b) & 1) << (3 * b + a)
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--skins", default="0,0.1,0.25,0.5,1.0")
    a = ap.parse_args()
    m, p = icp_amd.synthetic_pair(a.n, seed=42, angle_deg=5.0)
    lo, hi = m.min(0), m.max(0)
    h = np.cbrt(np.prod(hi - lo) * 2.0 / a.n)
    order = np.argsort(morton(p, lo, hi), kind="stable")
    p = p[order]
    tree = cKDTree(m)
    skins = [float(s) for s in a.skins.split(",")]
    _, idx = tree.query(p)
    q = p.copy()
    R = {s: np.zeros(a.n) for s in skins}  # (the first search: no certificate)
    print(f"n {a.n}, cell h {h:.4g}; per iteration: mean motion / h, NN changes, then per skin "
          f"(cells) walked queries and chunks with a walk")
    tot = {s: [0, 0] for s in skins}
    for it in range(1, a.iters):
        s_, Rm, t = fit(q, m[idx])
        qn = s_ * q @ Rm.T + t
        mot = np.sqrt(((qn - q) ** 2).sum(1))
        q = qn
        dd, ii = tree.query(q, k=2)
        e = np.sqrt(((q - m[idx]) ** 2).sum(1))  # the seed distance
        changed = ii[:, 0] != idx
        line = f"it {it:2d} motion/h {mot.mean() / h:.4f} changed {changed.mean():.4f}"
        for s in skins:
            Rs = R[s] - mot
            cert = e < Rs
            assert not np.any(cert & changed), "certificate wrong"
            walk = ~cert
            Rs = np.where(walk, np.minimum(dd[:, 1], e + s * h), Rs)
            R[s] = Rs
            wc = walk.reshape(-1, 32).any(1).mean() if a.n % 32 == 0 else float("nan")
            tot[s][0] += walk.mean()
            tot[s][1] += wc
            line += f" | {s}: {walk.mean():.3f} {wc:.3f}"
        idx = ii[:, 0]
        print(line, flush=True)
    n = a.iters - 1
    print("mean over seeded iterations: " + " | ".join(
        f"skin {s}: walked {tot[s][0] / n:.3f}, chunks {tot[s][1] / n:.3f}" for s in skins))


if __name__ == "__main__":
    main()
