"""The seeded grid search's fp32 prefilter bound (icp_grid.hip seeded_bound32, CPU restatement).

nn_grid_seeded32_kernel skips a point when its fp32 distance d32 = (dx^2 + dy^2) + dz^2 over the
offsets q32 = fl32(q - c), m32 = fl32(m - c) exceeds T = seeded_bound32(best, e): the claim is
that every model point with D64(q, m) <= best has d32 <= T, so no point that can be the first
minimum (or tie with it) is skipped.  Here the kernel's arithmetic is restated in numpy (float32
operations round like the GPU's with -ffp-contract=off) on adversarial sets: points on the seed's
sphere (exact and one-ulp ties), boxes far from the origin (large offsets), tiny and huge
extents, and queries outside the box.
"""
import numpy as np
import pytest


def em32(lo, hi):
    return np.ldexp(np.max(hi - lo), -23)


def bound32(best, e):
    s = np.sqrt(best) * (1.0 + 2.0 ** -50) + 1.7320508075688774 * e
    return np.float32(s * s * (1.0 + 2.0 ** -20)) * np.float32(1.0 + 2.0 ** -22)


def d64(q, m):
    d = q - m
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def d32(q, m, c):
    q32 = (q - c).astype(np.float32)
    m32 = (m - c).astype(np.float32)
    d = (q32 - m32).astype(np.float32)
    return ((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]).astype(np.float32) + d[..., 2] * d[..., 2]).astype(
        np.float32)


@pytest.mark.parametrize("centre,extent", [(0.0, 2.0), (1e3, 2.0), (-5e4, 10.0), (0.0, 2e-6), (7.0, 1e5)])
def test_points_at_least_as_close_as_the_seed_pass_the_bound(centre, extent):
    rng = np.random.default_rng(int(abs(centre) + extent * 1000) % (2**32))
    lo = np.full(3, centre - extent / 2)
    hi = np.full(3, centre + extent / 2)
    c = lo + 0.5 * (hi - lo)
    em = em32(lo, hi)
    fails = 0
    for _ in range(200):
        q = rng.uniform(lo - 0.1 * extent, hi + 0.1 * extent)
        r = extent * 10.0 ** rng.uniform(-5, -1)
        # the seed and many points on / just inside its sphere (ties to the last ulp)
        dirs = rng.normal(size=(400, 3))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        pts = q + r * dirs
        pts = np.clip(pts, lo, hi)
        seed = pts[0]
        best = d64(q, seed)
        dd = d64(q, pts)
        close = pts[dd <= best]
        o = q - c
        e = np.ldexp(np.max(np.abs(o)), -23) + em
        T = bound32(best, e)
        got = d32(q, close, c)
        fails += int(np.sum(got > T))
        # and the points one ulp inside: nudge towards q
        inner = q + np.nextafter(pts - q, 0.0)
        inner = np.clip(inner, lo, hi)
        di = d64(q, inner)
        close = inner[di <= best]
        fails += int(np.sum(d32(q, close, c) > T))
    assert fails == 0


def test_bound_is_tight_enough_to_prune():
    """Far points are skipped: at C4's scale the bound is a few ulps above the seed's distance."""
    rng = np.random.default_rng(1)
    lo, hi = np.full(3, -1.0), np.full(3, 1.0)
    c = np.zeros(3)
    q = rng.uniform(-1, 1, 3)
    best = 1e-4
    e = np.ldexp(np.max(np.abs(q - c)), -23) + em32(lo, hi)
    T = bound32(best, e)
    assert T < best * (1 + 1e-3)
    far = q + np.array([[0.0, 0.0, 0.0101]])  # D = 1.0201e-4 > best
    assert d32(q, far, c)[0] > T
