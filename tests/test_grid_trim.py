"""The seeded grid search's row trim (icp_grid.hip trim_row, CPU restatement).

nn_grid_seeded_kernel / nn_grid_seeded32_kernel scan, of each row (cy, cz) of a query's cell box,
only the x-cells trim_row leaves: the claim is that every model point m with D64(q, m) <= best
lies in a cell the trim keeps, so the first minimum and every point tied with it are still
scanned.  Here cell1 (fp64), the grid's cell assignment and trim_row's fp32 arithmetic in cell
units are restated in numpy (float32 operations round like the GPU's; sqrt is correctly rounded
here, and the kernel's 2^-18 factor covers a few ulps) and checked on adversarial sets: points on
and one ulp inside the seed's sphere, queries on cell boundaries and outside the grid, boxes far
from the origin, and grids at the 4,096-cell limit.
"""
import numpy as np
import pytest

F = np.float32


def cellt(t, g):
    t = np.asarray(t, dtype=np.float64)
    out = np.where(t >= g - 1, g - 1, np.floor(np.where(t > 0, t, 0.0))).astype(np.int64)
    return np.where(~(t > 0), 0, out)


def cell1(x, lo, inv_h, g):
    return cellt((x - lo) * inv_h, g)


def trim_row(q, best, lo, inv_h, g, cy, cz, x0, x1):
    """trim_row as the kernel computes it; returns (keep, x0, x1)."""
    t = (q - lo) * inv_h
    if np.any(np.abs(t) > 8192.0):
        return True, x0, x1
    tq = t.astype(F)
    sigma = F(2.0 ** -8)
    rho = F(np.sqrt(best) * inv_h) * F(1.0 + 2.0 ** -20)
    gap = []
    for a, c in ((1, cy), (2, cz)):
        d = F(0.0)
        if c <= g[a] - 2:
            d = max(d, F(tq[a] - F(c + 1)))
        if c >= 1:
            d = max(d, F(F(c) - tq[a]))
        gap.append(max(F(d - sigma), F(0.0)))
    rem = F(F(rho * rho) * F(1.0 + 2.0 ** -20)) - F(F(gap[0] * gap[0]) + F(gap[1] * gap[1]))
    if not rem >= 0:
        return False, x0, x1
    rx = F(np.sqrt(rem)) * F(1.0 + 2.0 ** -18)
    lo_t = F(F(tq[0] - rx) - sigma)
    hi_t = F(F(tq[0] + rx) + sigma)
    x0 = max(x0, int(cellt(float(lo_t), g[0])))
    x1 = min(x1, int(cellt(float(hi_t), g[0])))
    return x0 <= x1, x0, x1


def d64(q, m):
    d = q - m
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def check(q, pts, best, lo, inv_h, g):
    """Every point with D64 <= best is in a cell its row's trim keeps; returns the kept fraction."""
    cells = np.stack([cell1(pts[:, a], lo[a], inv_h, g[a]) for a in range(3)], axis=1)
    close = d64(q, pts) <= best
    kept_rows = {}
    for (cx, cy, cz), c in zip(cells, close):
        if (cy, cz) not in kept_rows:
            kept_rows[(cy, cz)] = trim_row(q, best, lo, inv_h, g, cy, cz, 0, g[0] - 1)
        keep, x0, x1 = kept_rows[(cy, cz)]
        if c:
            assert keep and x0 <= cx <= x1, (q, best, cx, cy, cz, x0, x1)
    return kept_rows


@pytest.mark.parametrize("centre,extent,g", [(0.0, 2.0, 64), (1e3, 2.0, 64), (-5e4, 10.0, 200),
                                             (0.0, 2e-6, 16), (7.0, 1e5, 4096), (0.5, 1.0, 3)])
def test_points_within_the_seed_distance_keep_their_cells(centre, extent, g):
    rng = np.random.default_rng(int(abs(centre) + extent * 1000 + g) % (2**32))
    lo = np.full(3, centre - extent / 2)
    gg = np.array([g, max(g // 2, 1), g])
    inv_h = (gg[0] - 0.5) / extent  # (g = floor(ext / h) + 1 cells along x)
    for _ in range(60):
        q = rng.uniform(lo - 0.05 * extent, lo + 1.05 * extent)
        if rng.random() < 0.3:  # a query on a cell boundary
            a = rng.integers(3)
            q[a] = lo[a] + rng.integers(0, gg[a]) / inv_h
        r = 10.0 ** rng.uniform(-1, 0.7) / inv_h
        dirs = rng.normal(size=(300, 3))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        pts = q + r * dirs
        seed = pts[0]
        best = d64(q, seed)
        inner = q + np.nextafter(pts - q, 0.0)  # one ulp inside
        check(q, np.concatenate([pts, inner, q[None, :]]), best, lo, inv_h, gg)


def test_trim_drops_corner_rows_and_narrows_runs():
    """It does trim: a query at a cell centre with a seed half a cell away keeps only its own
    row's middle run and the four edge-adjacent rows' middle cells, none of the corner rows."""
    g = np.array([10, 10, 10])
    lo, inv_h = np.zeros(3), 1.0
    q = np.array([5.5, 5.5, 5.5])
    best = 0.45 ** 2
    keep, x0, x1 = trim_row(q, best, lo, inv_h, g, 5, 5, 4, 6)
    assert keep and (x0, x1) == (5, 5)
    assert not trim_row(q, best, lo, inv_h, g, 4, 4, 4, 6)[0]  # corner row: gap^2 = 2 * 0.5^2 > 0.45^2
    keep, x0, x1 = trim_row(q, 0.6 ** 2, lo, inv_h, g, 4, 5, 4, 6)
    assert keep and (x0, x1) == (5, 5)
