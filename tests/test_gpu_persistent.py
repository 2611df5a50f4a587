"""The one-launch registration of small clouds (icp_set_run_mode, launch_icp_persistent).

For a single-rank icp_run of n <= 4096 scene points against a model that fits in LDS, the
engine runs the whole loop of GPU::ICP::find_corresponding_opti (src/GPU/gpu.cc:52-83) as ONE
launch of co-resident workgroups with one grid barrier per iteration.  Its sums are built from
the same per-thread partials and the same fold tree as the launch-per-step loop, so the two
must agree BIT FOR BIT: error trace, (s, R, t), final cloud and correspondences -- on the
bundled cow pair (converging and threshold-free runs), on random pairs whose sizes straddle
the single-workgroup pass boundaries (4, 255, 256, 257, ..., 4096 points; models from 1 to
6,000 points), with a NaN scene point, and in both NN modes.  The oracle trajectory is checked
too (rtol 1e-9, tests/golden/traces.json).
"""
import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def run(amd, m, p, mode, iters, threshold=1e-5, nn_mode=0, variant=0):
    with amd.Context(0, nn_mode) as ctx:
        ctx.set_nn_variant(variant)
        ctx.set_run_mode(mode)
        ctx.set_allow_unequal(m.shape[0] != p.shape[0])
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(iters, threshold)
        out = (res.iterations, res.converged, res.err, res.s, tuple(res.R), tuple(res.t), errs,
               ctx.get_scene(), ctx.get_indices(), ctx.stats()["persistent_runs"])
    return out


def assert_same(a, b):
    assert a[:6] == b[:6] or (np.isnan(a[2]) and np.isnan(b[2])), (a[:6], b[:6])
    np.testing.assert_array_equal(a[6], b[6])
    np.testing.assert_array_equal(a[7], b[7])
    np.testing.assert_array_equal(a[8], b[8])


@pytest.mark.parametrize("scene,iters,threshold", [("cow_tr1", 20, 1e-5), ("cow_tr2", 20, 1e-5),
                                                   ("cow_tr1", 1, -1.0), ("cow_tr1", 2, -1.0),
                                                   ("cow_tr2", 15, -1.0)])
@pytest.mark.parametrize("nn_mode", [0, 1])
def test_cow_one_launch_matches_launch_loop(amd, golden, scene, iters, threshold, nn_mode):
    m = amd.load_matrix(datasets.path("cow_ref"))
    p = amd.load_matrix(datasets.path(scene))
    one = run(amd, m, p, amd.RUN_PERSISTENT, iters, threshold, nn_mode)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, iters, threshold, nn_mode)
    auto = run(amd, m, p, amd.RUN_AUTO, iters, threshold, nn_mode)
    assert one[9] == 1 and loop[9] == 0 and auto[9] == 1  # the default takes the one launch
    assert_same(one, loop)
    assert_same(auto, loop)
    if threshold > 0:
        g = golden[scene]
        assert one[0] == g["iterations"]
        np.testing.assert_allclose(one[6], g["err"], rtol=1e-9)


SIZES = [(4, 4), (7, 1), (100, 3000), (255, 255), (256, 256), (257, 600), (1000, 1000),
         (2903, 50), (3000, 6000), (4095, 4096), (4096, 4096)]


@pytest.mark.parametrize("n,nm", SIZES)
def test_random_sizes_bitwise(amd, n, nm):
    rng = np.random.default_rng(n * 7919 + nm)
    m = rng.uniform(-1, 1, size=(nm, 3))
    a = rng.uniform(0.05, 0.3)
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    rot = np.eye(3) + np.sin(a) * k + (1 - np.cos(a)) * k @ k
    p = m[rng.integers(0, nm, n)] @ rot.T + rng.normal(scale=0.05, size=3) + rng.normal(scale=0.01, size=(n, 3))
    one = run(amd, m, p, amd.RUN_PERSISTENT, 6, -1.0)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 6, -1.0)
    assert one[9] == 1 and loop[9] == 0
    assert one[0] == 6
    assert_same(one, loop)


def test_nan_scene_point(amd):
    rng = np.random.default_rng(3)
    m = rng.uniform(-1, 1, size=(500, 3))
    p = m + 0.01
    p[17, 1] = np.nan
    one = run(amd, m, p, amd.RUN_PERSISTENT, 3, -1.0)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 3, -1.0)
    assert one[9] == 1
    assert one[8][17] == 0  # a NaN query's correspondence is index 0 (the reference's scan)
    assert one[0] == loop[0] == 3
    np.testing.assert_array_equal(one[6], loop[6])
    np.testing.assert_array_equal(one[7], loop[7])
    np.testing.assert_array_equal(one[8], loop[8])


def test_ineligible_runs_take_the_launch_loop(amd):
    rng = np.random.default_rng(4)
    m = rng.uniform(-1, 1, size=(5000, 3))
    p = rng.uniform(-1, 1, size=(49153, 3))  # n > 192 x 256: beyond the co-resident classic grid
    assert run(amd, m, p, amd.RUN_PERSISTENT, 2, -1.0)[9] == 0
    m = rng.uniform(-1, 1, size=(9000, 3))  # model beyond LDS (small kernel)
    assert run(amd, m, p[:3000], amd.RUN_PERSISTENT, 2, -1.0)[9] == 0
    m = rng.uniform(-1, 1, size=(65537, 3))  # model beyond 64 superblocks (mid-size kernel)
    assert run(amd, m, p[:5000], amd.RUN_PERSISTENT, 2, -1.0)[9] == 0
    m = rng.uniform(-1, 1, size=(3000, 3))  # an explicit NN variant keeps its own cascade under AUTO
    assert run(amd, m, p[:3000], amd.RUN_AUTO, 2, -1.0, variant=amd.VARIANT_GRID)[9] == 0


def test_repeated_runs_and_per_operation_calls(amd):
    """Two icp_run calls on one context continue from the resident scene; a closest_matrix
    afterwards still answers from the resident model."""
    m = amd.load_matrix(datasets.path("cow_ref"))
    p = amd.load_matrix(datasets.path("cow_tr2"))
    outs = {}
    for mode in (amd.RUN_PERSISTENT, amd.RUN_LAUNCHES):
        with amd.Context(0) as ctx:
            ctx.set_run_mode(mode)
            ctx.set_model(m)
            ctx.set_scene(p)
            r1, e1 = ctx.run(4, -1.0)
            r2, e2 = ctx.run(5, 1e-5)
            s = ctx.get_scene()
            _, idx = ctx.closest_matrix(s)
            outs[mode] = (e1, e2, r2.iterations, s, idx, ctx.stats()["persistent_runs"])
    a, b = outs[amd.RUN_PERSISTENT], outs[amd.RUN_LAUNCHES]
    assert a[5] == 2 and b[5] == 0
    for x, y in zip(a[:5], b[:5]):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("case", ["lattice_ties", "duplicates", "far_scene", "planar"])
def test_ties_and_degenerate_models_bitwise(amd, case):
    """The one-launch NN scans only the model blocks within each query's seed distance and
    breaks exact D64 ties by original index: lattice models with half-integer queries (many
    equidistant points), duplicated model points, a scene far outside the model (every block
    in range) and a planar model."""
    rng = np.random.default_rng(["lattice_ties", "duplicates", "far_scene", "planar"].index(case) + 50)
    if case == "lattice_ties":
        g = np.arange(-7, 8, dtype=float)
        m = np.stack(np.meshgrid(g, g, g[:8], indexing="ij"), axis=-1).reshape(-1, 3)
        m = m[rng.permutation(m.shape[0])]
        p = m[rng.integers(0, m.shape[0], 1500)] + 0.5  # equidistant from up to 8 lattice points
    elif case == "duplicates":
        base = rng.uniform(-1, 1, size=(700, 3))
        m = np.concatenate([base, base[::-1], base[:300]])
        m = m[rng.permutation(m.shape[0])]
        p = base[rng.integers(0, 700, 2000)] + rng.normal(scale=1e-3, size=(2000, 3))
    elif case == "far_scene":
        m = rng.uniform(-1, 1, size=(3000, 3))
        p = rng.uniform(-1, 1, size=(3000, 3)) + np.array([50.0, -20.0, 5.0])
    else:
        m = rng.uniform(-1, 1, size=(2500, 3))
        m[:, 2] = 0.25
        p = m[rng.integers(0, 2500, 2500)] + rng.normal(scale=0.02, size=(2500, 3))
        p[:, 2] = 0.25 + 0.1
    one = run(amd, m, p, amd.RUN_PERSISTENT, 5, -1.0)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 5, -1.0)
    assert one[9] == 1 and one[0] == 5
    assert_same(one, loop)


# ---- the fused iteration tail of mid-size runs (4,096 < n <= 49,152): one launch for moments,
# reduce, Horn, transform, reduce and error step, bit-identical to the six launches.  (Under
# AUTO an explicit NN variant keeps the launch loop, whose iterations end in the fused tail.) --


@pytest.mark.parametrize("pair,iters,threshold,nn_mode,variant", [
    (("horse_ref", "horse_tr1"), 50, 1e-5, 0, 3),   # C3 with the default cascade's f16 filter
    (("horse_ref", "horse_tr2"), 20, 1e-5, 0, 3),   # converges at 8
    (("bun000", "bun045"), 50, 1e-5, 0, 3),         # C2 (allow_unequal)
    (("bun000", "bun045"), 6, -1.0, 1, 3),          # fp64 NN
    (("horse_ref", "horse_tr1"), 6, -1.0, 0, 4),    # grid variant
])
def test_fused_tail_matches_launches(amd, pair, iters, threshold, nn_mode, variant):
    m = amd.load_matrix(datasets.path(pair[0]))
    p = amd.load_matrix(datasets.path(pair[1]))
    fused = run(amd, m, p, amd.RUN_AUTO, iters, threshold, nn_mode, variant)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, iters, threshold, nn_mode, variant)
    assert fused[9] == loop[9] == 0  # (not the one-launch registration: n > 4,096)
    assert_same(fused, loop)


@pytest.mark.parametrize("n,nm", [(4097, 4097), (8192, 3000), (12345, 20000), (49152, 49152)])
def test_fused_tail_random_sizes(amd, n, nm):
    rng = np.random.default_rng(n + 3 * nm)
    m = rng.normal(size=(nm, 3))
    p = m[rng.integers(0, nm, n)] @ np.array([[0.99, -0.1, 0.0], [0.1, 0.99, 0.0], [0.0, 0.0, 1.0]]).T + 0.03
    fused = run(amd, m, p, amd.RUN_AUTO, 7, -1.0, variant=amd.VARIANT_MFMA16)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 7, -1.0)
    assert fused[9] == 0 and fused[0] == 7
    assert_same(fused, loop)


# ---- the one-launch registration of mid-size runs (icp_persistent_mid_kernel): 4,096 < n <=
# 49,152 scene points, models up to 65,536 points in global memory; bit-identical to the loop --


@pytest.mark.parametrize("pair,iters,threshold,nn_mode", [
    (("horse_ref", "horse_tr1"), 50, 1e-5, 0),   # C3 as bench.py runs it
    (("horse_ref", "horse_tr2"), 20, 1e-5, 0),   # converges at 8
    (("bun000", "bun045"), 50, 1e-5, 0),         # C2 (allow_unequal)
    (("bun000", "bun045"), 6, -1.0, 1),          # fp64 NN mode in the loop
    (("horse_ref", "horse_tr1"), 1, -1.0, 0),    # one iteration: the first pass and the last residual
    (("horse_ref", "horse_tr1"), 2, -1.0, 0),
])
def test_mid_one_launch_matches_launch_loop(amd, golden, pair, iters, threshold, nn_mode):
    m = amd.load_matrix(datasets.path(pair[0]))
    p = amd.load_matrix(datasets.path(pair[1]))
    one = run(amd, m, p, amd.RUN_AUTO, iters, threshold, nn_mode)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, iters, threshold, nn_mode)
    assert one[9] == 1 and loop[9] == 0  # the default takes the one launch
    assert_same(one, loop)
    if threshold > 0 and pair[1] in golden:
        g = golden[pair[1]]
        assert one[0] == g["iterations"]
        np.testing.assert_allclose(one[6], g["err"], rtol=1e-9)


MID_SIZES = [(4097, 4097), (4097, 1), (5000, 64), (8192, 3000), (12345, 20000), (30000, 65536),
             (40000, 40000), (49152, 49152)]


@pytest.mark.parametrize("n,nm", MID_SIZES)
def test_mid_random_sizes_bitwise(amd, n, nm):
    rng = np.random.default_rng(n * 31 + nm)
    m = rng.uniform(-1, 1, size=(nm, 3))
    a = rng.uniform(0.05, 0.3)
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    rot = np.eye(3) + np.sin(a) * k + (1 - np.cos(a)) * k @ k
    p = m[rng.integers(0, nm, n)] @ rot.T + rng.normal(scale=0.05, size=3) + rng.normal(scale=0.01, size=(n, 3))
    one = run(amd, m, p, amd.RUN_PERSISTENT, 6, -1.0)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 6, -1.0)
    assert one[9] == 1 and loop[9] == 0
    assert one[0] == 6
    assert_same(one, loop)


@pytest.mark.parametrize("case", ["lattice_ties", "duplicates", "far_scene", "planar", "nan_point"])
def test_mid_ties_and_degenerate_models_bitwise(amd, case):
    """The mid-size kernel's culled scan (superblocks, then blocks) on the small kernel's hard
    cases at 4,096 < n: exact ties broken by original index, duplicated points, a scene far
    outside the model, a planar model and a NaN scene point (index 0)."""
    rng = np.random.default_rng(["lattice_ties", "duplicates", "far_scene", "planar", "nan_point"].index(case) + 90)
    if case == "lattice_ties":
        g = np.arange(-12, 13, dtype=float)
        m = np.stack(np.meshgrid(g, g, g[:12], indexing="ij"), axis=-1).reshape(-1, 3)
        m = m[rng.permutation(m.shape[0])]
        p = m[rng.integers(0, m.shape[0], 9000)] + 0.5  # equidistant from up to 8 lattice points
    elif case == "duplicates":
        base = rng.uniform(-1, 1, size=(3000, 3))
        m = np.concatenate([base, base[::-1], base[:1000]])
        m = m[rng.permutation(m.shape[0])]
        p = base[rng.integers(0, 3000, 8000)] + rng.normal(scale=1e-3, size=(8000, 3))
    elif case == "far_scene":
        m = rng.uniform(-1, 1, size=(6000, 3))
        p = rng.uniform(-1, 1, size=(6000, 3)) + np.array([50.0, -20.0, 5.0])
    elif case == "planar":
        m = rng.uniform(-1, 1, size=(20000, 3))
        m[:, 2] = 0.25
        p = m[rng.integers(0, 20000, 20000)] + rng.normal(scale=0.02, size=(20000, 3))
        p[:, 2] = 0.25 + 0.1
    else:
        m = rng.uniform(-1, 1, size=(10000, 3))
        p = m + 0.01
        p[4321, 1] = np.nan
    one = run(amd, m, p, amd.RUN_PERSISTENT, 4, -1.0)
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 4, -1.0)
    assert one[9] == 1 and one[0] == 4
    if case == "nan_point":
        assert one[8][4321] == 0  # a NaN query's correspondence is index 0 (the reference's scan)
        for x, y in zip(one[6:9], loop[6:9]):
            np.testing.assert_array_equal(x, y)
    else:
        assert_same(one, loop)


def test_mid_repeated_runs_and_per_operation_calls(amd):
    m = amd.load_matrix(datasets.path("horse_ref"))
    p = amd.load_matrix(datasets.path("horse_tr2"))
    outs = {}
    for mode in (amd.RUN_PERSISTENT, amd.RUN_LAUNCHES):
        with amd.Context(0) as ctx:
            ctx.set_run_mode(mode)
            ctx.set_model(m)
            ctx.set_scene(p)
            r1, e1 = ctx.run(3, -1.0)
            r2, e2 = ctx.run(10, 1e-5)
            s = ctx.get_scene()
            _, idx = ctx.closest_matrix(s)
            outs[mode] = (e1, e2, r2.iterations, s, idx, ctx.stats()["persistent_runs"])
    a, b = outs[amd.RUN_PERSISTENT], outs[amd.RUN_LAUNCHES]
    assert a[5] == 2 and b[5] == 0
    for x, y in zip(a[:5], b[:5]):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("pair", [("cow_ref", "cow_tr1"), ("horse_ref", "horse_tr2")])
def test_first_barrier_abort_falls_back_to_the_launch_loop(amd, pair, monkeypatch):
    """A one-launch run whose grid is not co-resident (another persistent kernel holding CUs)
    gives up at its first grid barrier, before it writes any state, and icp_run takes the launch
    loop: the same results, counted in persistent_fallbacks.  ICP_PERSIST_TEST_ABORT=1 makes the
    first barrier fail at once; a later run on the same context takes the one launch again (its
    barrier words were reset)."""
    m = amd.load_matrix(datasets.path(pair[0]))
    p = amd.load_matrix(datasets.path(pair[1]))
    loop = run(amd, m, p, amd.RUN_LAUNCHES, 20, 1e-5)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        monkeypatch.setenv("ICP_PERSIST_TEST_ABORT", "1")
        res, errs = ctx.run(20, 1e-5)
        st = ctx.stats()
        assert st["persistent_runs"] == 0 and st["persistent_fallbacks"] == 1
        assert res.iterations == loop[0]
        np.testing.assert_array_equal(errs, loop[6])
        np.testing.assert_array_equal(ctx.get_scene(), loop[7])
        np.testing.assert_array_equal(ctx.get_indices(), loop[8])
        monkeypatch.delenv("ICP_PERSIST_TEST_ABORT")
        ctx.set_scene(p)
        res2, errs2 = ctx.run(20, 1e-5)
        assert ctx.stats()["persistent_runs"] == 1
        np.testing.assert_array_equal(errs2, loop[6])
        np.testing.assert_array_equal(ctx.get_scene(), loop[7])


def test_fused_tail_barrier_abort_reruns_with_launches(amd, monkeypatch):
    """the launch loop's fused mid-size tail (moments ... error step in one
    launch, 4,096 < n <= 49,152) has grid barriers too.  If one times out (its workgroups not all
    co-resident), icp_run restores the scene and correspondences it started from and runs the
    registration again with the separate launches.  ICP_PERSIST_TEST_ABORT=1 keeps the one-launch
    kernel out (the run falls back to the loop, whose tails are then fused) and
    ICP_TAIL_TEST_ABORT=1 fails the first tail's first barrier: the result must be the launch
    loop's, bit for bit, and a second run on the same context (seeded by its correspondences)
    must match the loop's second run too."""
    m = amd.load_matrix(datasets.path("horse_ref"))
    p = amd.load_matrix(datasets.path("horse_tr1"))
    with amd.Context(0) as ctx:
        ctx.set_run_mode(amd.RUN_LAUNCHES)
        ctx.set_model(m)
        ctx.set_scene(p)
        ref1 = ctx.run(12, -1.0)
        s1, i1 = ctx.get_scene(), ctx.get_indices()
        ref2 = ctx.run(5, -1.0)
        s2, i2 = ctx.get_scene(), ctx.get_indices()
    monkeypatch.setenv("ICP_PERSIST_TEST_ABORT", "1")
    monkeypatch.setenv("ICP_TAIL_TEST_ABORT", "1")
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(12, -1.0)
        assert res.iterations == ref1[0].iterations
        np.testing.assert_array_equal(errs, ref1[1])
        np.testing.assert_array_equal(ctx.get_scene(), s1)
        np.testing.assert_array_equal(ctx.get_indices(), i1)
        res, errs = ctx.run(5, -1.0)
        np.testing.assert_array_equal(errs, ref2[1])
        np.testing.assert_array_equal(ctx.get_scene(), s2)
        np.testing.assert_array_equal(ctx.get_indices(), i2)


def test_randomised_bitwise_fuzz(amd):
    """tools/persist_fuzz.py, a short run: random sizes over both one-launch kernels' ranges,
    uniform / surface / clustered / lattice (exact ties) / duplicated models, small to far
    motions, fixed or converging runs -- every case one launch and bit-identical to the loop
    (6,000 cases of it: profiles/r02bg_persist_fuzz/)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "persist_fuzz", os.path.join(os.path.dirname(__file__), "..", "tools", "persist_fuzz.py"))
    fz = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fz)
    rng = np.random.default_rng(2024)
    kinds = ["uniform", "surface", "clusters", "lattice", "duplicates"]
    for c in range(60):
        small = c % 3 == 0
        n = int(rng.integers(4, 4097)) if small else int(rng.integers(4097, 49153))
        nm = int(rng.integers(1, 6001)) if small else int(rng.integers(16, 65537))
        kind = kinds[c % len(kinds)]
        m = fz.model(rng, kind, nm)
        p = fz.rigid(rng, m[rng.integers(0, nm, n)] + rng.normal(scale=0.01, size=(n, 3)), [0.2, 1.0, 10.0][c % 3])
        if kind == "lattice":
            p = np.round(p * 2) / 2 + 0.5
        iters, thr = int(rng.integers(1, 9)), (-1.0 if c % 2 else 1e-6)
        one = fz.run(m, p, amd.RUN_PERSISTENT, iters, thr)
        loop = fz.run(m, p, amd.RUN_LAUNCHES, iters, thr)
        assert one[4] == 1 and loop[4] == 0, (c, n, nm, kind)
        assert one[0] == loop[0], (c, n, nm, kind)
        for x, y in zip(one[1:4], loop[1:4]):
            np.testing.assert_array_equal(x, y, err_msg=f"case {c}: n={n} nm={nm} {kind}")


@pytest.mark.parametrize("variant", ["auto", "bundle"])
def test_scale_fuzz_certified_equals_fp64(amd, variant):
    """tools/scale_fuzz.py, a short run: the default cascade of the launch loop (f16 MFMA filter,
    certificate, grid resolver, fp64 fallback) against the fp64 brute force at 2^15..2^19 points,
    every model shape of persist_fuzz, rescaled and offset clouds; unseeded and seeded iterations
    bit for bit (error trace, final cloud, per-iteration correspondence digests).  Longer runs:
    profiles/r02s3g/."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "scale_fuzz", os.path.join(os.path.dirname(__file__), "..", "tools", "scale_fuzz.py"))
    sf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sf)
    rng = np.random.default_rng(77)
    kinds = ["uniform", "surface", "clusters", "lattice", "duplicates"]
    queued = 0
    for c in range(10):
        n, nm = int(2 ** rng.uniform(15, 18)), int(2 ** rng.uniform(15, 18))
        kind = kinds[c % len(kinds)]
        m = sf.model(rng, kind, nm)
        p = sf.rigid(rng, m[rng.integers(0, nm, n)] + rng.normal(scale=0.01, size=(n, 3)), [0.2, 1.0, 10.0][c % 3])
        if kind == "lattice":
            p = np.round(p * 2) / 2 + 0.5
        else:
            sc, off = 10.0 ** rng.uniform(-3, 3), rng.normal(size=3) * 100.0
            m, p = m * sc + off * sc, p * sc + off * sc
        cert = sf.run(m, p, amd.NN_CERTIFIED, 3, amd.VARIANT_BUNDLE if variant == "bundle" else amd.VARIANT_AUTO)
        ref = sf.run(m, p, amd.NN_FP64, 3)
        assert cert[0] == ref[0] == 3, (c, n, nm, kind)
        for x, y in zip(cert[1:4], ref[1:4]):
            np.testing.assert_array_equal(x, y, err_msg=f"case {c}: n={n} nm={nm} {kind}")
        queued += cert[4]["level1_queued"]
    assert queued > 0  # the grid resolver took part
