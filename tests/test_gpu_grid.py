"""The grid resolver (icp_grid.hip): exact fp64 first-minimum for the certificate's near ties.

Every certified variant hands its uncertified queries, with its fp32 winner as candidate, to
the uniform-grid resolver; boxes over the cell budget go back to the brute-force levels.
Indices must equal the oracle's (src/cpu.cc rule on squared fp64 distances, lowest index on
ties) bit for bit, whatever the shape of the model's bounding box.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(2024)
CERTIFIED = {"valu": 1, "mfma": 2, "mfma16": 3, "grid": 4}


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def search(amd, variant, m, p):
    with amd.Context(0, amd.NN_CERTIFIED) as ctx:
        ctx.set_nn_variant(CERTIFIED[variant])
        ctx.set_model(m)
        ctx.reset_stats()
        _, idx = ctx.closest_matrix(p)
        return idx, ctx.stats()


def integer_lattice(n):
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij"), -1)
    return g.reshape(-1, 3).astype(np.float64)


@pytest.mark.parametrize("variant", list(CERTIFIED))
def test_grid_flat_model(amd, oracle, variant):
    # all model points in the plane z = 0.25 (flat bounding box) on a half-integer lattice:
    # many exactly equidistant candidates
    xy = RNG.integers(0, 80, size=(6000, 2)) * 0.5
    m = np.column_stack([xy, np.full(len(xy), 0.25)])
    p = np.column_stack([RNG.integers(0, 160, size=(3000, 2)) * 0.25, RNG.uniform(-1, 1, 3000)])
    idx, _ = search(amd, variant, m, p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)


@pytest.mark.parametrize("variant", list(CERTIFIED))
def test_grid_line_and_identical_points(amd, oracle, variant):
    t = RNG.integers(0, 400, size=5000) * 0.125
    m = np.column_stack([t, 2.0 * t, -t])              # a line: two degenerate axes
    p = np.column_stack([t[:2000] + 0.0625, 2.0 * t[:2000], -t[:2000]]) + RNG.normal(scale=1e-3, size=(2000, 3))
    idx, _ = search(amd, variant, m, p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)
    same = np.tile([[1.5, -2.0, 3.0]], (777, 1))       # one point repeated: index 0 always
    idx, _ = search(amd, variant, same, RNG.normal(size=(300, 3)))
    assert (idx == 0).all()


@pytest.mark.parametrize("variant", list(CERTIFIED))
def test_grid_clustered_model(amd, oracle, variant):
    # two dense clusters 1e3 apart plus sparse outliers: most cells empty, a few crowded
    a = RNG.normal(scale=0.01, size=(20000, 3))
    b = RNG.normal(scale=0.01, size=(20000, 3)) + 1000.0
    o = RNG.uniform(-50, 1050, size=(200, 3))
    m = np.round(np.concatenate([a, b, o]) * 4096) / 4096   # coarse values: many ties
    p = np.round(np.concatenate([a[:3000] + 0.003, b[:3000] - 0.002, o[:100] + 1.0]) * 4096) / 4096
    idx, _ = search(amd, variant, m, p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)


@pytest.mark.parametrize("variant", list(CERTIFIED))
def test_grid_ties_over_budget_fall_back_to_brute_force(amd, oracle, variant):
    # hollow 60^3 lattice cube (faces only) and queries near its centre, tied between points
    # of several faces: the candidate ball spans the whole grid (> budget cells), so these
    # queries go back to the brute-force levels; queries near the faces stay in the grid
    g = integer_lattice(60)
    m = g[(g == 0).any(1) | (g == 59).any(1)]
    k = 48
    centre = np.column_stack([np.full(k, 29.5), np.full(k, 29.5), 29.5 + RNG.integers(-3, 4, k)])
    near = np.column_stack([np.full(k, 0.5), RNG.integers(1, 58, k) + 0.5, RNG.integers(1, 58, k) + 0.5])
    p = np.concatenate([centre, near])
    idx, st = search(amd, variant, m, p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)
    assert st["grid_fallback"] > 0, st


def test_grid_takes_the_near_ties_at_c4(amd):
    # at the bench configuration the grid must settle (almost) all level-1 leftovers
    m, p = amd.synthetic_pair(1 << 18, seed=7)
    idx, st = search(amd, "mfma16", m, p)
    assert st["level1_queued"] > 0, st
    assert st["grid_fallback"] <= max(16, st["level1_queued"] // 1000), st


def test_grid_variant_at_c4_matches_fp64_and_rarely_falls_back(amd):
    m, p = amd.synthetic_pair(1 << 18, seed=11)
    idx, st = search(amd, "grid", m, p)
    with amd.Context(0, amd.NN_FP64) as ctx:
        ctx.set_model(m)
        _, ref = ctx.closest_matrix(p)
    np.testing.assert_array_equal(idx, ref)
    assert st["grid_fallback"] <= 16, st


def icp_runs(amd, m, p, iters, variants=("grid", "fp64")):
    out = {}
    for name in variants:
        mode, variant = (amd.NN_FP64, 0) if name == "fp64" else (amd.NN_CERTIFIED, CERTIFIED[name])
        with amd.Context(0, mode) as ctx:
            ctx.set_nn_variant(variant)
            ctx.set_allow_unequal(m.shape[0] != p.shape[0])
            ctx.set_model(m)
            ctx.set_scene(p)
            ctx.reset_stats()
            res, errs = ctx.run(iters, -1.0)
            out[name] = (res, errs, ctx.get_scene(), ctx.get_indices(), ctx.stats())
    return out


def assert_same_run(runs, ref="fp64"):
    r0, e0, s0, i0, _ = runs[ref]
    for name, (r, e, s, i, _) in runs.items():
        assert r.iterations == r0.iterations, name
        np.testing.assert_array_equal(e, e0, err_msg=name)
        np.testing.assert_array_equal(s, s0, err_msg=name)
        np.testing.assert_array_equal(i, i0, err_msg=name)


def test_grid_variant_icp_run_hollow_cube_falls_back(amd):
    """icp_run with the grid variant: iterations >= 2 take the seeded resolve
    (launch_nn_grid_resolve_all).  On the hollow cube the scene's centre queries are tied
    across faces, their boxes exceed the budget and go to nn_resolve (T = +inf); the run must
    equal the fp64 brute force bit for bit."""
    g = integer_lattice(40)
    m = g[(g == 0).any(1) | (g == 39).any(1)]
    k = 600
    p = np.concatenate([np.column_stack([np.full(k, 19.5), np.full(k, 19.5), 19.5 + RNG.integers(-2, 3, k)]),
                        m[RNG.integers(0, m.shape[0], m.shape[0] - k)] + RNG.normal(scale=0.05, size=(m.shape[0] - k, 3))])
    runs = icp_runs(amd, m, p, 4)
    assert_same_run(runs)
    assert runs["grid"][4]["grid_fallback"] > 0, runs["grid"][4]


def test_grid_variant_icp_run_clustered(amd):
    a = RNG.normal(scale=0.01, size=(15000, 3))
    b = RNG.normal(scale=0.01, size=(15000, 3)) + 100.0
    m = np.round(np.concatenate([a, b]) * 4096) / 4096
    p = np.round((m[RNG.permutation(m.shape[0])[:20000]] + [0.002, -0.001, 0.0005]) * 4096) / 4096
    runs = icp_runs(amd, m, p, 5, ("grid", "mfma16", "valu", "fp64"))
    assert_same_run(runs)


def test_grid_variant_seeded_non_finite_scene_point(amd):
    """A NaN scene point makes the whole iteration non-finite (as in the reference).  The
    seeded grid resolve must still return the first-minimum rule's index for it (0: no
    comparison holds), like every other path, instead of keeping its stale seed."""
    m = RNG.normal(size=(5000, 3))
    p = m[RNG.integers(0, 5000, 5000)] + RNG.normal(scale=0.01, size=(5000, 3))
    p[17] = [np.nan, 0.0, 0.0]
    runs = icp_runs(amd, m, p, 3, ("grid", "valu", "fp64"))
    for name, (res, errs, scene, idx, _) in runs.items():
        assert res.iterations == 3, name
        assert np.isnan(errs).all(), name
        assert (idx == 0).all(), name  # every query is NaN after the first transform
    assert_same_run({k: (v[0], v[1], v[2], v[3], v[4]) for k, v in runs.items()})
