"""The fused grid iteration's sphere prune and exclusion certificate (icp_grid.hip
nn_grid_iter_kernel, CPU restatement).

Prune (ICP_ITER_PRUNE).  The walk scans, of a query's complete cell box [c0, c1] for the squared
radius ew, only the rows whose (y, z) slab reaches the sphere of radius sqrt(ew) and, of those,
only the x-cells of the sphere's chord -- computed in fp32 relative to the box's first cell with
room for every rounding.  The claim: every model point m with D64(q, m) <= ew lies in a kept row,
inside its kept x-run, so no point that can be the first minimum (or tie with it) is missed.
The kernel's arithmetic (tr, rcf, rc2, xroom, xspan, the row's (ry, rz) by an fp32 reciprocal,
dy, dz, rem, xw, the floor / clamp) is restated below in numpy float32 (rounding like the GPU's
with -ffp-contract=off; the square root is taken two ulps low, below any GPU rounding of it) and
checked on adversarial sets: points on and one ulp inside the sphere, queries on cell faces and
outside the grid, boxes 1e3..5e4 from the origin, grids of 4,096 cells a side.  A negative control
removes the room and finds misses.

Certificate.  A walked query's bound R = min(sqrt(ew) (1 - 2^-40), sqrt(a) (1 - 2^-20) - sqrt(3)
eq (1 + 2^-20)) over the smallest "other" value a (an fp32 distance d32, or a D64 rounded down),
lowered each iteration by the query's motion: Rc = (R - mot (1 + 2^-40)) - R 2^-48.  The claims
-- each bound is below the true distance (exact rational arithmetic here), and a certified
query's kept correspondence is the brute-force first minimum -- are checked on far-offset boxes,
lattices full of exact ties and trajectories of small rigid motions.
"""
import math
from fractions import Fraction

import numpy as np
import pytest

F = np.float32
SQRT3 = 1.7320508075688774


# ---- the grid's fp64 cell arithmetic (icp_gridbox.h) --------------------------------------------
def cellt(t, g):
    if not t > 0.0:
        return 0
    if t >= g - 1:
        return g - 1
    return int(t)


def cell1(x, lo, inv_h, g):
    return cellt((x - lo) * inv_h, g)


def complete_box(q, r2, lo, inv_h, g):
    R = math.sqrt(r2)
    c0, c1 = [0, 0, 0], [0, 0, 0]
    for a in range(3):
        s = (abs(q[a]) + R) * 2.0 ** -44
        c0[a] = cell1(q[a] - (R + s), lo[a], inv_h, g[a])
        c1[a] = cell1(q[a] + (R + s), lo[a], inv_h, g[a])
    return c0, c1


def d64(q, m):
    d = np.asarray(q, dtype=np.float64) - np.asarray(m, dtype=np.float64)
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def sqrtf_low(x):
    """sqrtf, then two ulps toward zero (a GPU square root may round either way by an ulp)."""
    r = np.sqrt(F(x))
    return np.nextafter(np.nextafter(r, F(0)), F(0))


# ---- the prune (icp_grid.hip, ICP_ITER_PRUNE block of nn_grid_iter_kernel) ----------------------
def prune_rows(q, ew, lo, inv_h, c0, c1, room=1.0):
    """{(ry, rz): (x0, x1)} of the rows the walk keeps, as the kernel computes them."""
    tr = [F((q[a] - lo[a]) * inv_h - float(c0[a])) for a in range(3)]
    rcf = F(math.sqrt(ew) * inv_h * (1.0 + 2.0 ** -18 * room) +
            2.0 ** -20 * room * (1.0 + abs(float(tr[0])) + abs(float(tr[1])) + abs(float(tr[2]))))
    rc2 = F(rcf * rcf)
    xroom = F(F(2.0 ** -20 * room) * F(F(1.0) + abs(tr[0])))
    xspan = F(c1[0] - c0[0] + 1)
    ny, nz = c1[1] - c0[1] + 1, c1[2] - c0[2] + 1
    inv_ny = F(F(1.0) / F(ny))
    rows = {}
    for r in range(ny * nz):
        rz = int(F(F(F(r) + F(0.5)) * inv_ny))
        ry = r - rz * ny
        assert (ry, rz) == (r % ny, r // ny)  # (the reciprocal's claim, exhaustively below)
        dy = max(F(0.0), max(F(F(ry) - tr[1]), F(tr[1] - F(ry + 1))))
        dz = max(F(0.0), max(F(F(rz) - tr[2]), F(tr[2] - F(rz + 1))))
        rem = F(F(rc2 - F(dy * dy)) - F(dz * dz))
        if rem < F(0.0):
            continue
        xw = F(F(sqrtf_low(rem) * F(1.0 + 2.0 ** -20 * room)) + xroom)
        x0 = max(c0[0], c0[0] + int(math.floor(max(F(tr[0] - xw), F(-1.0)))))
        x1 = min(c1[0], c0[0] + int(math.floor(min(F(tr[0] + xw), xspan))))
        if x0 <= x1:
            rows[(ry, rz)] = (x0, x1)
    return rows


def misses(q, pts, ew, lo, inv_h, g, room=1.0):
    """Points with D64(q, m) <= ew that the box or the prune would not scan."""
    c0, c1 = complete_box(q, ew, lo, inv_h, g)
    rows = prune_rows(q, ew, lo, inv_h, c0, c1, room)
    bad = 0
    for m in pts[d64(q, pts) <= ew]:
        c = [cell1(m[a], lo[a], inv_h, g[a]) for a in range(3)]
        if not all(c0[a] <= c[a] <= c1[a] for a in range(3)):
            bad += 1
            continue
        run = rows.get((c[1] - c0[1], c[2] - c0[2]))
        if run is None or not run[0] <= c[0] <= run[1]:
            bad += 1
    return bad


def adversarial_cases(centre, extent, gx, seed, n_q=40):
    """(q, pts, ew, lo, inv_h, g): queries on cell faces / outside the grid, points on the
    sphere and one ulp inside it, the radius from a fraction of a cell to several cells."""
    rng = np.random.default_rng(seed)
    g = [gx, max(gx // 3, 1), gx]
    lo = [centre - extent / 2] * 3
    inv_h = (gx - 0.5) / extent
    for _ in range(n_q):
        q = rng.uniform(np.array(lo) - 0.05 * extent, np.array(lo) + 1.05 * extent)
        if rng.random() < 0.5:  # on a cell face (one or two axes)
            for a in rng.choice(3, size=rng.integers(1, 3), replace=False):
                q[a] = lo[a] + rng.integers(0, g[a]) / inv_h
        r = 10.0 ** rng.uniform(-1.0, 0.5) / inv_h
        dirs = rng.normal(size=(250, 3))
        dirs[:6] = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]])
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        pts = q + r * dirs
        if rng.random() < 0.5:  # the sphere's x-extreme exactly on a cell face: the chord ends there
            k = math.floor((q[0] + r - lo[0]) * inv_h)
            face = lo[0] + k / inv_h
            if face > q[0]:
                pts[0] = [face, q[1], q[2]]
                r = face - q[0]
                pts[1:] = q + r * dirs[1:]
        ew = float(np.max(d64(q, pts)))  # every sphere point is within ew; most exactly on it
        inner = q + np.nextafter(pts - q, 0.0)
        # (model points lie in the grid's box -- the model's bounding box: a query may not)
        hi = [lo[a] + (g[a] - 0.5) / inv_h for a in range(3)]
        pts = np.concatenate([pts, inner])
        pts = pts[np.all((pts >= lo) & (pts <= hi), axis=1)]
        yield q, pts, ew, lo, inv_h, g


@pytest.mark.parametrize("centre,extent,gx", [(0.0, 2.0, 80), (1e3, 2.0, 64), (-5e4, 10.0, 200), (5e4, 3.0, 97),
                                              (7.0, 1e5, 4096), (0.0, 2e-6, 16), (0.5, 1.0, 3)])
def test_pruned_walk_keeps_every_point_within_the_radius(centre, extent, gx):
    total = 0
    for k, (q, pts, ew, lo, inv_h, g) in enumerate(adversarial_cases(centre, extent, gx, seed=gx + k_seed(centre))):
        total += misses(q, pts, ew, lo, inv_h, g)
    assert total == 0


def k_seed(c):
    return int(abs(c)) % 9973


def test_negative_control_without_room_misses_points():
    """The test can fail: with the room removed, points on the sphere fall outside the fp32 chord."""
    total = 0
    for centre, extent, gx in ((1e3, 2.0, 64), (-5e4, 10.0, 200), (0.0, 2.0, 80)):
        for q, pts, ew, lo, inv_h, g in adversarial_cases(centre, extent, gx, seed=gx + 1, n_q=60):
            total += misses(q, pts, ew, lo, inv_h, g, room=0.0)
    assert total > 0


def test_prune_drops_rows_and_narrows_runs():
    """It does prune: a query at a cell centre keeps, of its 3 x 3 x 3 box, only the rows and
    cells its sphere reaches."""
    g, lo, inv_h = [10, 10, 10], [0.0] * 3, 1.0
    q = [5.5, 5.5, 5.5]
    c0, c1 = complete_box(q, 0.45 ** 2, lo, inv_h, g)
    assert (c0, c1) == ([5, 5, 5], [5, 5, 5])  # the box itself is one cell
    c0, c1 = [4, 4, 4], [6, 6, 6]  # a 3 x 3 x 3 box around it, as a larger seed would give
    assert prune_rows(q, 0.45 ** 2, lo, inv_h, c0, c1) == {(1, 1): (5, 5)}  # the neighbours: 0.5 away
    # radius 0.6: the own row's whole run, the edge-adjacent rows' middle cell, no corner row
    # (0.5^2 + 0.5^2 > 0.6^2)
    rows = prune_rows(q, 0.6 ** 2, lo, inv_h, c0, c1)
    assert rows == {(1, 1): (4, 6), (0, 1): (5, 5), (2, 1): (5, 5), (1, 0): (5, 5), (1, 2): (5, 5)}


def test_row_reciprocal_is_exact():
    """(r + 0.5) / ny by an fp32 reciprocal gives r // ny for every row of a box of up to 2^12
    rows and ny <= 125 (the walk's boxes: at most kSeededBox = 125 cells)."""
    for ny in range(1, 126):
        inv_ny = F(F(1.0) / F(ny))
        r = np.arange(4096, dtype=np.int64)
        rz = ((r.astype(F) + F(0.5)).astype(F) * inv_ny).astype(F).astype(np.int64)
        assert np.array_equal(rz, r // ny), ny


# ---- the certificate's bounds -------------------------------------------------------------------
def em32(lo, hi):
    return math.ldexp(max(h - l for l, h in zip(lo, hi)), -23)


def d32(q, m, c):
    q32 = np.array([F(q[a] - c[a]) for a in range(3)])
    m32 = np.array([F(m[a] - c[a]) for a in range(3)])
    d = (q32 - m32).astype(F)
    return F(F(F(d[0] * d[0]) + F(d[1] * d[1])) + F(d[2] * d[2]))


def exact_d2(q, m):
    return sum((Fraction(float(q[a])) - Fraction(float(m[a]))) ** 2 for a in range(3))


def bound_from(a, eq):
    return math.sqrt(float(a)) * (1.0 - 2.0 ** -20) - SQRT3 * eq * (1.0 + 2.0 ** -20)


def below(b, d2):
    """b <= sqrt(d2) exactly (b a double, d2 a Fraction)."""
    return b <= 0.0 or Fraction(b) ** 2 <= d2


@pytest.mark.parametrize("centre,extent", [(0.0, 2.0), (1e3, 2.0), (-5e4, 10.0), (7.0, 1e5), (0.0, 2e-6)])
def test_other_bounds_are_below_the_true_distance(centre, extent):
    rng = np.random.default_rng(int(abs(centre) + extent) % 9973)
    lo = [centre - extent / 2] * 3
    hi = [centre + extent / 2] * 3
    c = [l + 0.5 * (h - l) for l, h in zip(lo, hi)]
    em = em32(lo, hi)
    worst = 0.0
    for _ in range(300):
        q = rng.uniform(np.array(lo) - 0.1 * extent, np.array(hi) + 0.1 * extent)
        r = extent * 10.0 ** rng.uniform(-7, -1)
        m = np.clip(q + r * rng.normal(size=3) / math.sqrt(3), lo, hi)
        eq = math.ldexp(max(abs(q[a] - c[a]) for a in range(3)), -23) + em
        true2 = exact_d2(q, m)
        a32 = d32(q, m, c)
        b = bound_from(a32, eq)
        assert below(b, true2), (q, m, a32, eq)
        a64 = np.float32(np.nextafter(F(d64(q, m)), F(0)))  # __double2float_rd(D64): at most this
        b = bound_from(max(a64, F(0)), eq)
        assert below(b, true2)
        if b > 0:
            worst = max(worst, b / math.sqrt(float(true2)))
    assert worst < 1.0


def test_motion_bound_rounds_up():
    """The kernel's fp32 motion bound is at least the exact |q' - q| (the fp64 square rounded up to
    fp32, its v_sqrt_f32 root -- taken two ulps low here -- times 1 + 2^-21), over motions from
    1e-12 to 1e3."""
    rng = np.random.default_rng(9)
    for _ in range(3000):
        q = rng.uniform(-1e4, 1e4, 3)
        d = rng.normal(size=3)
        d *= 10.0 ** rng.uniform(-12, 3) / np.linalg.norm(d)
        qn = q + d
        m = motion_bound(q, qn)
        r = np.float32(m / (1.0 + 2.0 ** -21))
        m_low = float(np.nextafter(np.nextafter(r, F(0)), F(0))) * (1.0 + 2.0 ** -21)  # (v_sqrt_f32 two ulps low)
        assert Fraction(min(m, m_low)) ** 2 >= exact_d2(q, qn)


def test_motion_decrement_rounds_down():
    """Rc = (R - mot (1 + 2^-40)) - R 2^-48 is at most the exact R - |q' - q|, even in near
    cancellation (mot within an ulp of R)."""
    rng = np.random.default_rng(5)
    for _ in range(2000):
        R = float(np.float32(10.0 ** rng.uniform(-6, 2)))
        q = rng.uniform(-1e3, 1e3, 3)
        d = rng.normal(size=3)
        d *= R * (1.0 - 10.0 ** rng.uniform(-15, 0)) / np.linalg.norm(d)
        q2 = q + d
        mot = math.sqrt(float(d64(q, q2)))
        Rc = (R - mot * (1.0 + 2.0 ** -40)) - R * 2.0 ** -48
        true_mot2 = exact_d2(q, q2)
        if Rc > 0:
            # Rc + |q' - q| <= R  <=>  |q' - q| <= R - Rc
            assert Fraction(R) - Fraction(Rc) >= 0 and (Fraction(R) - Fraction(Rc)) ** 2 >= true_mot2


# ---- the certificate over a trajectory (state machine against brute force) ----------------------
def f32_rd(x):
    """__double2float_rd: the largest float32 <= x."""
    f = np.float32(x)
    return float(np.nextafter(f, F(-np.inf))) if float(f) > x else float(f)


def state_bound(r):
    return f32_rd(r) if r > 0 else -1.0


def walk(q, pts, seed, lo, inv_h, g, c, em, skin, two=True):
    """A walk of nn_grid_iter2_kernel for one query: the exact first minimum over the scanned
    points and the next state (R1, R3, winner, second point).  Every scanned point other than the
    winner is an "other" with its d32 (the kernel's lanes mix in D64 rounded down for candidates;
    both bound from below); R1 bounds every point but the winner, R3 every point outside the pair."""
    e = float(d64(q, pts[seed]))
    rs = math.sqrt(e) + skin
    ew = rs * rs
    c0, c1 = complete_box(q, ew, lo, inv_h, g)
    rows = prune_rows(q, ew, lo, inv_h, c0, c1)
    cells = np.array([[cell1(p[a], lo[a], inv_h, g[a]) for a in range(3)] for p in pts])
    scanned = []
    for j, cc in enumerate(cells):
        run = rows.get((cc[1] - c0[1], cc[2] - c0[2]))
        if all(c0[a] <= cc[a] <= c1[a] for a in range(3)) and run and run[0] <= cc[0] <= run[1]:
            scanned.append(j)
    scanned = np.array(scanned)
    dd = d64(q, pts[scanned])
    order = np.lexsort((scanned, dd))
    win = int(scanned[order[0]])
    eq = math.ldexp(max(abs(q[a] - c[a]) for a in range(3)), -23) + em
    others = sorted((float(d32(q, pts[j], c)), int(j)) for j in scanned if j != win)
    u0 = math.sqrt(ew) * (1.0 - 2.0 ** -40)

    def lower(k):
        return min(u0, bound_from(others[k][0], eq)) if len(others) > k else u0

    r1, r3 = lower(0), (lower(1) if two else -1.0)
    h2 = others[0][1] if two and others else -1
    return win, h2, state_bound(r1), state_bound(r3)


def motion_bound(q, qn):
    """The kernel's motion: the fp64 square rounded up to fp32, its fp32 root, times 1 + 2^-21."""
    m2 = float(d64(q, qn))
    m2f = np.float32(m2)
    if float(m2f) < m2:
        m2f = np.nextafter(m2f, F(np.inf))
    return float(np.float32(np.sqrt(m2f) * F(1.0 + 2.0 ** -21)))


def inside(d2, r):
    return r > 0.0 and d2 * (1.0 + 2.0 ** -38) < r * r * (1.0 - 2.0 ** -50)


def certify(qn, pts, st, mot, two):
    """The kernel's phase-A certificate: (winner, next state) or None (the query walks)."""
    h, h2, R1, R3 = st
    if not (R1 > 0 or R3 > 0):
        return None
    R1c = (R1 - mot) - R1 * 2.0 ** -48
    R3c = (R3 - mot) - R3 * 2.0 ** -48
    e = float(d64(qn, pts[h]))
    if inside(e, R1c):
        return h, (h, h2, state_bound(R1c), state_bound(R3c))
    if two and h2 >= 0 and R3c > 0:
        d2 = float(d64(qn, pts[h2]))
        swap = d2 < e or (d2 == e and h2 < h)
        if inside(d2 if swap else e, R3c):
            lb = min(R3c, math.sqrt(e if swap else d2) * (1.0 - 2.0 ** -40))
            if swap:
                return h2, (h2, h, state_bound(lb), state_bound(R3c))
            return h, (h, h2, state_bound(max(R1c, lb)), state_bound(R3c))
    return None


def first_min(q, pts):
    dd = d64(q, pts)
    return int(np.lexsort((np.arange(len(pts)), dd))[0])


def rot(axis, deg):
    a = np.asarray(axis, dtype=np.float64)
    a /= np.linalg.norm(a)
    t = math.radians(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(t) * K + (1 - math.cos(t)) * K @ K


@pytest.mark.parametrize("model,two", [("lattice", True), ("lattice", False), ("jitter", True), ("far", True)])
def test_certified_queries_keep_the_first_minimum(model, two):
    rng = np.random.default_rng({"lattice": 1, "jitter": 2, "far": 3}[model] + (0 if two else 10))
    k = 12
    ax = np.arange(k, dtype=np.float64)
    pts = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)  # exact ties everywhere
    if model == "jitter":
        pts = pts + rng.uniform(-0.3, 0.3, pts.shape)
    if model == "far":
        pts = pts * 0.01 + 3e4
    lo = pts.min(0).tolist()
    hi = pts.max(0).tolist()
    ext = max(h - l for l, h in zip(lo, hi))
    inv_h = 1.0 / (ext / (k - 1) * 1.3)
    g = [int(math.floor((h - l) * inv_h)) + 1 for l, h in zip(lo, hi)]
    c = [l + 0.5 * (h - l) for l, h in zip(lo, hi)]
    em = em32(lo, hi)
    skin = 0.25 / inv_h
    step = ext / (k - 1)
    nq = 60
    q = np.array(lo) + step * rng.uniform(2, k - 3, (nq, 3))
    q[: nq // 3] = np.round(q[: nq // 3] / step * 2) * step / 2  # on bisector planes: exact ties
    q[: nq // 3] += np.array(lo) - np.round(np.array(lo) / step * 2) * step / 2
    state = [walk(qq, pts, first_min(qq, pts), lo, inv_h, g, c, em, skin, two) for qq in q]
    certified = 0
    centre = q.mean(0)
    for it in range(12):
        Rm = rot((1, 2, 3), rng.uniform(-0.4, 0.4))
        tmv = rng.normal(size=3) * step * 10.0 ** rng.uniform(-4, -1.5)
        qn = (q - centre) @ Rm.T + centre + tmv
        for i in range(nq):
            got = certify(qn[i], pts, state[i], motion_bound(q[i], qn[i]), two)
            if got is not None:
                assert got[0] == first_min(qn[i], pts), (model, it, i)
                certified += 1
                state[i] = got[1]
            else:
                state[i] = walk(qn[i], pts, state[i][0], lo, inv_h, g, c, em, skin, two)
                assert state[i][0] == first_min(qn[i], pts)
        q = qn
    assert certified > 0  # (the certificate does fire on these trajectories)


def test_far_count_shortcut_is_exact():
    """nn_grid_iter2_kernel counts a query far (its complete box over 125 cells) only when e inv_h^2
    >= 2.2: below that the box spans at most 4 cells an axis.  Checked against complete_box on
    seed distances just under the cut, queries on and off cell faces, boxes far from the origin."""
    rng = np.random.default_rng(13)
    for centre, g in ((0.0, 80), (1e3, 64), (-5e4, 200)):
        lo = [centre - 1.0] * 3
        inv_h = (g - 0.5) / 2.0
        gg = [g, g, g]
        for _ in range(3000):
            q = rng.uniform(np.array(lo) - 0.1, np.array(lo) + 2.1)
            if rng.random() < 0.5:
                a = rng.integers(3)
                q[a] = lo[a] + rng.integers(0, g) / inv_h
            e = 2.2 * (1.0 - 10.0 ** rng.uniform(-15, 0)) / (inv_h * inv_h)
            if not e * (inv_h * inv_h) < 2.2:
                continue
            c0, c1 = complete_box(q, e, lo, inv_h, gg)
            cells = (c1[0] - c0[0] + 1) * (c1[1] - c0[1] + 1) * (c1[2] - c0[2] + 1)
            assert cells <= 64, (q, e, cells)
