"""The fused grid iteration (icp_grid.hip nn_grid_iter2_kernel: the pending transform, the
exclusion certificate, the packed walks, the moments) on adversarial scenes against the oracle's
brute force (cpu.cc:5-27's first minimum, oracle closest_blocked).

Every case has a model and a scene of >= 2^16 points (the slot-order path) and runs the GRID
variant, so a run's first search is the seeded pass from cell seeds and every later one the
fused kernel.  run(k) on one context gives iteration k's indices -- the fused kernel's, each query
certified or walked -- and run(k - 1) on a fresh context the scene they were searched on (the
trajectory is exact, so it is the same scene); 1,024 sampled queries are checked against the
brute force, and the runs must have certified queries (the certificate was exercised):

  lattice   a 41^3 integer lattice model, the scene the lattice offset by (0.5, 0.5, 0.25) and
            turned a degree: every query near-equidistant from two to eight model points, at
            every iteration
  boundary  a uniform cube model; a third of the scene beyond the model's box (up to two grid
            cells past a face: clamped border cells), a third exactly on the box's faces
  shell     a hollow lattice cube (faces only, mostly empty cells) and a scene inside and
            outside it: long walks through empty cells, ties across the shell
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SAMPLE = 1024


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def rotation(deg, axis=(1.0, 2.0, 3.0)):
    a = np.asarray(axis) / np.linalg.norm(axis)
    t = np.deg2rad(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def lattice(n):
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij"), -1)
    return g.reshape(-1, 3).astype(np.float64)


def case(name):
    rng = np.random.default_rng(11)
    if name == "lattice":
        m = lattice(41)
        c = m.mean(axis=0)
        p = (m + [0.5, 0.5, 0.25] - c) @ rotation(1.0).T + c
    elif name == "boundary":
        n = 1 << 16
        m = rng.uniform(-1.0, 1.0, size=(n, 3))
        p = m @ rotation(2.0).T + [0.01, -0.02, 0.015]
        k = n // 3
        h = np.cbrt(8.0 * 2.0 / n)  # (about the grid's cell: two points a cell)
        axis = rng.integers(0, 3, size=k)
        side = rng.choice([-1.0, 1.0], size=k)
        p[np.arange(k), axis] = side * (1.0 + rng.uniform(0.0, 2.0 * h, size=k))  # beyond a face
        axis2 = rng.integers(0, 3, size=k)
        lo, hi = m.min(axis=0), m.max(axis=0)
        p[k + np.arange(k), axis2] = np.where(rng.random(k) < 0.5, lo[axis2], hi[axis2])  # on the box's faces
    else:  # shell
        g = lattice(60)
        m = g[np.any((g == 0) | (g == 59), axis=1)]  # 60^3's faces: 20,888 points
        m = np.concatenate([m, m + 0.5 * (rng.random(m.shape) < 0.5)])  # ties and near ties: 41,776
        m = np.concatenate([m, m[: (1 << 16) - len(m)] + [0.25, 0.25, 0.0]])
        p = rng.uniform(-3.0, 62.0, size=(1 << 16, 3))
        p = (p - 29.5) @ rotation(1.5).T + 29.5
    return m, p


def indices_after(amd, m, p, k):
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(amd.VARIANT_GRID)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(k, -1.0)
        return ctx.get_indices(), ctx.stats()


def scene_after(amd, m, p, k):
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(amd.VARIANT_GRID)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(k, -1.0)
        return ctx.get_scene()


@pytest.mark.parametrize("name", ["lattice", "boundary", "shell"])
def test_fused_iteration_matches_brute_force(amd, oracle, name):
    m, p = case(name)
    assert len(m) >= 1 << 16 and len(p) >= 1 << 16
    sel = np.sort(np.random.default_rng(7).choice(len(p), SAMPLE, replace=False))
    certified = 0
    for k in (2, 4, 7):
        got, st = indices_after(amd, m, p, k)
        assert st["run_grid_searches"] == k, st
        certified += st["run_certified"]
        cur = scene_after(amd, m, p, k - 1)
        _, ref = oracle.closest_blocked(cur[sel], m)
        assert np.array_equal(got[sel], ref), (name, k, int(np.sum(got[sel] != ref)))
    assert certified > 0  # the certificate settled queries in these runs


def test_certificate_counts_accumulate_over_runs(amd):
    """The certificate's per-strand counts stay on the device across runs of one scene size (no
    synchronisation at a run's start), fold into the stats at a size change, and reset with them."""
    n = 1 << 17
    m, p = amd.synthetic_pair(n, seed=5)
    m2, p2 = amd.synthetic_pair(n // 2 + 77, seed=6)
    def counts(st):
        return st["run_certified"], st["run_walked"]
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(amd.VARIANT_GRID)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(6, -1.0)
        one = counts(ctx.stats())
        assert one[0] > 0 and one[1] > 0
        ctx.set_scene(p)
        ctx.run(6, -1.0)
        assert counts(ctx.stats()) == (2 * one[0], 2 * one[1])
        with amd.Context(0) as c2:  # another size: its counts alone
            c2.set_nn_variant(amd.VARIANT_GRID)
            c2.set_model(m2)
            c2.set_scene(p2)
            c2.run(6, -1.0)
            small = counts(c2.stats())
        ctx.set_model(m2)
        ctx.set_scene(p2)
        ctx.run(6, -1.0)  # (a size change: the first two runs' counts fold into the stats)
        assert counts(ctx.stats()) == (2 * one[0] + small[0], 2 * one[1] + small[1])
        ctx.reset_stats()
        assert counts(ctx.stats()) == (0, 0)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(6, -1.0)
        assert counts(ctx.stats()) == one
