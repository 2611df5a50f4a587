"""HIP path vs the CPU oracle (parity tests proper; run on an MI355X with -m gpu).

Tolerances:
  * NN indices: bit-exact (index work) — both NN modes, every dataset, every edge case;
  * per-iteration err: rel 1e-9; s, R: abs 1e-9; t and final new_p: abs 1e-9 x extent
    on the bundled clouds (fp64 throughout; reduction order is the only difference);
  * ICP_NN_FP64 and ICP_NN_CERTIFIED runs are bitwise identical to each other.
"""
import json
import os

import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
RNG = np.random.default_rng(99)
# (nn_mode, filter variant): certified with the VALU filter, certified with the MFMA filter
# (+ VALU second level + fp64), fp64 brute force
# (+ "bundle": the f16 filter behind the per-(query, bundle) bound, for models >= 8192 points)
MODES = ["valu", "mfma", "mfma16", "grid", "bundle", "fp64"]
_MODE_ARGS = {"valu": (0, 1), "mfma": (0, 2), "mfma16": (0, 3), "grid": (0, 4), "bundle": (0, 5), "fp64": (1, 0)}


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


@pytest.fixture(scope="module")
def ctxs(amd):
    c = {}
    for m in MODES:
        c[m] = amd.Context(0, _MODE_ARGS[m][0])
        c[m].set_nn_variant(_MODE_ARGS[m][1])
    yield c
    for v in c.values():
        v.close()


def load(amd, name):
    return amd.load_matrix(datasets.path(name))


def gold_npz(name):
    return np.load(os.path.join(GOLD, f"{name}_oracle.npz"))


@pytest.fixture(scope="module")
def golden_traces():
    with open(os.path.join(GOLD, "traces.json")) as f:
        return json.load(f)


# ---- NN: bit-exact indices -------------------------------------------------------------

@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("cfg", ["cow_tr1", "cow_tr2", "horse_tr1", "horse_tr2", "bunny"])
def test_nn_iteration0_matches_fixture(amd, ctxs, golden_traces, mode, cfg):
    g = golden_traces[cfg]
    m, p = load(amd, g["model"]), load(amd, g["scene"])
    ctx = ctxs[mode]
    ctx.set_model(m)
    y, idx = ctx.closest_matrix(p)
    ref = gold_npz(cfg)["idx0"]
    assert np.array_equal(idx, ref), f"{int((idx != ref).sum())} mismatches"
    np.testing.assert_array_equal(y, m[ref])


def test_nn_synthetic_fixture(amd, ctxs):
    z = np.load(os.path.join(GOLD, "synthetic4096.npz"))
    for mode in MODES:
        ctxs[mode].set_model(z["model"])
        _, idx = ctxs[mode].closest_matrix(z["scene"])
        np.testing.assert_array_equal(idx, z["idx0"])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("np_,nm", [(1, 1), (1, 5), (5, 1), (3, 1023), (257, 1024), (1000, 1025),
                                    (4097, 3000), (300000, 2048), (2048, 300001)])
def test_nn_random_sizes(amd, ctxs, oracle, mode, np_, nm):
    m = RNG.uniform(-3, 3, size=(nm, 3)) + np.array([10.0, -5.0, 2.0])
    p = RNG.uniform(-3, 3, size=(np_, 3)) + np.array([10.0, -5.0, 2.0])
    ctx = ctxs[mode]
    ctx.set_model(m)
    _, idx = ctx.closest_matrix(p)
    sel = np.arange(np_) if np_ * nm <= 4e8 else RNG.choice(np_, size=int(4e8 // nm), replace=False)
    _, ref = oracle.closest(p[sel], m)
    np.testing.assert_array_equal(idx[sel], ref)


@pytest.mark.parametrize("mode", MODES)
def test_nn_exact_ties_and_duplicates(amd, ctxs, oracle, mode):
    # integer grid: many exactly equidistant model points + duplicated model points
    g = np.stack(np.meshgrid(np.arange(12), np.arange(12), np.arange(12), indexing="ij"), -1).reshape(-1, 3)
    m = np.concatenate([g, g[::7], g[::3]]).astype(np.float64) * 0.5
    p = (RNG.integers(0, 23, size=(5000, 3)) * 0.25).astype(np.float64)
    ctx = ctxs[mode]
    ctx.set_model(m)
    _, idx = ctx.closest_matrix(p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)


@pytest.mark.parametrize("variant", [1, 2, 3])
def test_nn_certificate_sends_ties_to_resolution(amd, variant):
    with amd.Context(0, 0) as ctx:
        ctx.set_nn_variant(variant)
        m = np.array([[1.0, 0, 0], [-1.0, 0, 0], [0, 1.0, 0], [5, 5, 5.0]])
        ctx.set_model(m)
        ctx.reset_stats()
        _, idx = ctx.closest_matrix(np.array([[0.0, 0, 0], [4.0, 4, 4]]))
        assert idx.tolist() == [0, 3]


@pytest.mark.parametrize("mode", MODES)
def test_nn_far_offset_cloud(amd, ctxs, oracle, mode):
    # coordinates ~1e6 away from the origin: the fp32 filter works on centred values
    m = RNG.normal(size=(5000, 3)) + 1.0e6
    p = RNG.normal(size=(3000, 3)) + 1.0e6
    ctxs[mode].set_model(m)
    _, idx = ctxs[mode].closest_matrix(p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)


def test_nn_certified_equals_fp64_at_1m(amd, ctxs, oracle):
    m, p = amd.synthetic_pair(1 << 20, seed=42)
    out = {}
    for mode in MODES:
        ctxs[mode].set_model(m)
        ctxs[mode].reset_stats()
        _, out[mode] = ctxs[mode].closest_matrix(p)
    np.testing.assert_array_equal(out["valu"], out["fp64"])
    np.testing.assert_array_equal(out["mfma"], out["fp64"])
    np.testing.assert_array_equal(out["mfma16"], out["fp64"])
    np.testing.assert_array_equal(out["grid"], out["fp64"])
    np.testing.assert_array_equal(out["bundle"], out["fp64"])
    sel = RNG.choice(p.shape[0], size=96, replace=False)
    _, ref = oracle.closest(p[sel], m)
    np.testing.assert_array_equal(out["fp64"][sel], ref)


@pytest.mark.parametrize("variant", [2, 3, 5])
def test_mfma_level1_certifies_most_queries(amd, variant):
    # the MFMA filters recover their argmin by recomputing G (f32: VALU fma chain, f16:
    # re-running the MFMA); if those bits ever differed, the queries would all fall back to
    # level 2.  On random data almost every query must be settled at level 1 or 2.
    m, p = amd.synthetic_pair(1 << 17, seed=3)
    with amd.Context(0, 0) as ctx:
        ctx.set_nn_variant(variant)
        ctx.set_model(m)
        ctx.set_scene(p, np_total=p.shape[0])
        ctx.set_allow_unequal(True)
        ctx.run(1, -1.0)
        st = ctx.stats()
    assert st["level1_queued"] < 0.1 * p.shape[0], st
    assert st["ambiguous"] < 0.01 * p.shape[0], st


# ---- full ICP loop vs oracle trajectories ----------------------------------------------

def run_engine(amd, mode, m, p, max_iter, threshold, allow_unequal=False):
    with amd.Context(0, _MODE_ARGS[mode][0]) as ctx:
        ctx.set_nn_variant(_MODE_ARGS[mode][1])
        ctx.set_allow_unequal(allow_unequal)
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(max_iter, threshold)
        return res, errs, ctx.get_scene()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("cfg", ["cow_tr1", "cow_tr2", "horse_tr2", "horse_tr1", "bunny"])
def test_icp_trajectory_matches_oracle(amd, golden_traces, mode, cfg):
    g = golden_traces[cfg]
    m, p = load(amd, g["model"]), load(amd, g["scene"])
    res, errs, new_p = run_engine(amd, mode, m, p, g["max_iter"], g["threshold"], g["allow_unequal"])
    assert res.iterations == g["iterations"]
    rtol = 1e-3 if cfg == "bunny" else 1e-9  # bunny: tie-sensitive trajectory
    np.testing.assert_allclose(errs, g["err"], rtol=rtol)
    np.testing.assert_allclose(np.array(res.R).reshape(3, 3), np.array(g["R"][-1]), atol=1e-9 if cfg != "bunny" else 1e-3)
    assert res.s == pytest.approx(g["s"][-1], abs=1e-9 if cfg != "bunny" else 1e-3)
    extent = float(np.abs(m).max())
    ref_p = gold_npz(cfg)["new_p"]
    np.testing.assert_allclose(new_p, ref_p, atol=(1e-9 if cfg != "bunny" else 1e-3) * extent)


def test_icp_synthetic_fixed_iterations(amd, golden_traces):
    g = golden_traces["synthetic4096"]
    z = np.load(os.path.join(GOLD, "synthetic4096.npz"))
    res, errs, new_p = run_engine(amd, "mfma", z["model"], z["scene"], 30, -1.0)
    assert res.iterations == 30 and not res.converged
    np.testing.assert_allclose(errs, g["err"], rtol=1e-9)
    np.testing.assert_allclose(new_p, z["new_p"], atol=1e-9)


def test_modes_bitwise_identical(amd):
    m, p = load(amd, "horse_ref"), load(amd, "horse_tr1")
    a = run_engine(amd, "valu", m, p, 6, -1.0)
    for mode in ("mfma", "mfma16", "grid", "bundle", "fp64"):
        b = run_engine(amd, mode, m, p, 6, -1.0)
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[2], b[2])


def test_reference_fatal_checks(amd):
    m = RNG.normal(size=(10, 3))
    with amd.Context(0, 0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(m[:9])
        with pytest.raises(amd.ICPError) as ei:
            ctx.run(5)
        assert ei.value.code == amd.ICP_E_SIZE_MISMATCH
        ctx.set_model(m[:3])
        ctx.set_scene(m[:3])
        with pytest.raises(amd.ICPError) as ei:
            ctx.run(5)
        assert ei.value.code == amd.ICP_E_TOO_FEW_POINTS
        with pytest.raises(amd.ICPError):
            amd.Context(0, 0).run(3)  # no model


def test_zero_iterations_leaves_scene(amd):
    m = RNG.normal(size=(100, 3))
    res, errs, new_p = run_engine(amd, "valu", m, m + 0.1, 0, 1e-5)
    assert res.iterations == 0 and errs.size == 0
    np.testing.assert_array_equal(new_p, m + 0.1)


# ---- per-operation surface (src/GPU/gpu.hh:110-116) ------------------------------------

def test_surface_ops_match_oracle(amd, oracle):
    m, p = load(amd, "cow_ref"), load(amd, "cow_tr2")
    y, _ = oracle.closest(p, m)
    al = oracle.find_alignment(p, y)
    with amd.Context(0, 0) as ctx:
        mu, centred = ctx.compute_centroid(p)
        np.testing.assert_allclose(mu, np.array(al.mu_p), rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(centred, p - mu, atol=0)
        d_caps, sp = ctx.y_p_norm(y - np.array(al.mu_y), p - np.array(al.mu_p))
        assert d_caps == pytest.approx(al.d_caps, rel=1e-12)
        assert sp == pytest.approx(al.sp, rel=1e-12)
        s, R, t, e = ctx.find_alignment(p, y)
        assert s == pytest.approx(al.s, rel=1e-12)
        np.testing.assert_allclose(R, np.array(al.R).reshape(3, 3), atol=1e-12)
        np.testing.assert_allclose(t, np.array(al.t), atol=1e-12)
        assert e == pytest.approx(al.err, rel=1e-9)
        sR = (al.s * np.array(al.R)).reshape(9)
        e1, p_same = ctx.err_compute(y, p, False, sR, al.t)
        np.testing.assert_array_equal(p_same, p)
        e2, p_new = ctx.err_compute(y, p, True, sR, al.t)
        oe, op = oracle.err_compute(p, y, al.s, al.R, al.t)
        assert e1 == e2 and e2 == pytest.approx(oe, rel=1e-12)
        np.testing.assert_array_equal(p_new, op)  # per-point transform bitwise = oracle


@pytest.mark.parametrize("n", [1, 2, 3, 4, 255, 256, 257, 2903, 4095, 4096, 4097, 10000])
def test_surface_ops_across_the_single_workgroup_boundary(amd, oracle, n):
    """The per-operation calls take one launch on mapped memory up to 4,096 points and the
    multi-workgroup passes above: both against the oracle on random clouds of every size class,
    the per-point transform bitwise.  (find_alignment from 3 points: with 1 point the scale is
    0 / 0 on every path, with 2 the rotation about their line is undetermined.)"""
    rng = np.random.default_rng(n)
    p = rng.normal(size=(n, 3)) * 3.0 + 1.0
    y = p @ np.array([[0.96, -0.28, 0.0], [0.28, 0.96, 0.0], [0.0, 0.0, 1.0]]).T + 0.3 + rng.normal(scale=0.01, size=(n, 3))
    al = oracle.find_alignment(p, y)
    with amd.Context(0, 0) as ctx:
        mu, centred = ctx.compute_centroid(p)
        np.testing.assert_allclose(mu, p.mean(axis=0), rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(centred, p - mu, atol=0)
        if n >= 3:
            s, R, t, e = ctx.find_alignment(p, y)
            assert s == pytest.approx(al.s, rel=1e-10)
            np.testing.assert_allclose(R, np.array(al.R).reshape(3, 3), atol=1e-10)
            np.testing.assert_allclose(t, np.array(al.t), atol=1e-9)
            assert e == pytest.approx(al.err, rel=1e-8, abs=1e-12)
        sc, R0, t0 = 1.01, [0.96, -0.28, 0.0, 0.28, 0.96, 0.0, 0.0, 0.0, 1.0], [0.1, -0.2, 0.3]
        sR = (sc * np.array(R0)).reshape(9)
        e1, p_same = ctx.err_compute(y, p, False, sR, t0)
        np.testing.assert_array_equal(p_same, p)
        e2, p_new = ctx.err_compute(y, p, True, sR, t0)
        oe, op = oracle.err_compute(p, y, sc, R0, t0)
        assert e1 == e2 and e2 == pytest.approx(oe, rel=1e-11, abs=1e-12)
        np.testing.assert_array_equal(p_new, op)  # per-point transform bitwise = oracle


def test_reference_shaped_icp_class(amd, golden_traces):
    m, p = load(amd, "cow_ref"), load(amd, "cow_tr1")
    icp = amd.ICP(m, p, 20)
    res = icp.find_corresponding_opti()
    assert res.iterations == 7 and res.converged
    np.testing.assert_allclose(icp.errors, golden_traces["cow_tr1"]["err"], rtol=1e-9)
    np.testing.assert_allclose(icp.new_p, m, atol=1e-5)


def test_naive_path_matches_opti_and_oracle(amd, golden_traces):
    # GPU::ICP::find_corresponding_naive (gpu.cc:17-49): one NN call per point; the same
    # NN rule as the batched search, so the same 7-iteration trajectory on cow
    m, p = load(amd, "cow_ref"), load(amd, "cow_tr1")
    icp = amd.ICP(m, p, 20)
    it = icp.find_corresponding_naive()
    assert it == 7
    np.testing.assert_allclose(icp.errors, golden_traces["cow_tr1"]["err"], rtol=1e-9)
    np.testing.assert_allclose(icp.new_p, m, atol=1e-5)
    sel = RNG.choice(p.shape[0], size=64, replace=False)
    _, ref = amd.compute_Y_w_opti(m, p)
    for j in sel:
        assert amd.compute_distance_w_naive(m, p[j]) == ref[j]


@pytest.mark.parametrize("nq", [1, 7, 32, 33])
def test_nn_few_queries_exact(amd, oracle, nq):
    """<= 32 queries under the automatic variant take the one-launch exact path (the per-point
    API); 33 take the certified cascade.  Both are the oracle's first minimum, ties included."""
    m = np.floor(RNG.uniform(-4, 4, size=(3000, 3)))  # integer lattice points: many exact ties
    p = np.floor(RNG.uniform(-4, 4, size=(nq, 3))) + 0.5
    with amd.Context(0, amd.NN_CERTIFIED) as ctx:
        ctx.set_model(m)
        y, idx = ctx.closest_matrix(p)
    _, ref = oracle.closest(p, m)
    np.testing.assert_array_equal(idx, ref)
    np.testing.assert_array_equal(y, m[ref])


@pytest.mark.parametrize("mode", MODES)
def test_nn_non_finite_and_far_queries(amd, ctxs, oracle, mode):
    """NaN, +-inf and astronomically far queries must neither fault nor return an index outside
    the model (a NaN query gets index 0, what the reference's GPU scan returns when no
    comparison holds); the finite queries beside them keep their exact answers."""
    m = RNG.normal(size=(3000, 3))
    good = RNG.normal(size=(200, 3))
    bad = np.array([[np.nan, 0, 0], [np.inf, 0, 0], [-np.inf, 1, 1], [1e30, 0, 0], [-1e20, 5, 5],
                    [np.nan, np.nan, np.nan], [0, 0, np.inf], [3e18, -3e18, 1e18]])
    p = np.concatenate([good, bad, good[:50]])
    ctxs[mode].set_model(m)
    _, idx = ctxs[mode].closest_matrix(p)
    assert idx.min() >= 0 and idx.max() < m.shape[0]
    _, ref = oracle.closest(good, m)
    np.testing.assert_array_equal(idx[:200], ref)
    np.testing.assert_array_equal(idx[208:], ref[:50])
    # few-query path (automatic variant, <= 32 queries)
    with amd.Context(0, amd.NN_CERTIFIED) as ctx:
        ctx.set_model(m)
        _, idx_few = ctx.closest_matrix(bad)
    assert idx_few.min() >= 0 and idx_few.max() < m.shape[0]


def test_icp_degenerate_scene_does_not_fault(amd):
    """All scene points identical: sum ||p'||^2 = 0, so Horn's scale is infinite and the next
    iterations search with non-finite queries (the reference computes the same inf/NaN).  The
    run must complete and report, not fault."""
    m = RNG.normal(size=(5000, 3))
    p = np.tile([[0.3, -0.2, 0.1]], (5000, 1))
    with amd.Context(0, amd.NN_CERTIFIED) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(5)
        out = ctx.get_scene()
    assert res.iterations == 5
    assert out.shape == p.shape


@pytest.mark.parametrize("seed", range(10))
def test_paths_bitwise_consistent_random(amd, seed):
    """Random scenes whose sizes straddle the engine's path thresholds (fused small tail at
    n <= 4096, f16 MFMA filter at 8192, model larger/smaller than the scene): every certified
    filter variant must follow the fp64 brute-force trajectory bit for bit (errs and final
    scene), since each certifies the reference's exact first minimum.  (Sizes up to ~50k run
    the r4 f16 plan, 131,072 the r8 one.)"""
    rng = np.random.default_rng(1000 + seed)
    n = [7, 300, 4096, 4097, 8191, 8192, 12000, 20000, 65536, 131072][seed]
    nm = int(rng.choice([n, max(4, n // 2), n + 1000]))
    m = rng.normal(size=(nm, 3)) if seed % 3 == 0 else rng.uniform(-1, 1, size=(nm, 3))
    if seed % 3 == 2:
        m[:, 2] *= 1e-3  # nearly planar model: many near ties
    a = rng.uniform(0.02, 0.3)
    axis = rng.normal(size=3); axis /= np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    rot = np.eye(3) + np.sin(a) * k + (1 - np.cos(a)) * k @ k
    p = m[rng.integers(0, nm, n)] @ rot.T + rng.normal(scale=0.05, size=3) \
        + rng.normal(scale=0.01, size=(n, 3))
    runs = {}
    for name, (mode, variant) in list(_MODE_ARGS.items()) + [("auto", (0, 0))]:
        with amd.Context(0, mode) as ctx:
            ctx.set_nn_variant(variant)
            ctx.set_allow_unequal(n != nm)
            ctx.set_model(m)
            ctx.set_scene(p)
            res, errs = ctx.run(8, -1.0)
            runs[name] = (res.iterations, errs, ctx.get_scene())
    ref_it, ref_errs, ref_scene = runs["fp64"]
    assert ref_it == 8
    for name, (it, errs, scene) in runs.items():
        assert it == ref_it, name
        np.testing.assert_array_equal(errs, ref_errs, err_msg=name)
        np.testing.assert_array_equal(scene, ref_scene, err_msg=name)
