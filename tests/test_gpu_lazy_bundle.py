"""The bundle filter's images built at their first use, and what icp_run's transforms hand to the
next search (icp_engine.hip: build_bundle / ensure_bundle, run_loop's SeedState and records_args;
icp_step.hip: transform_err_kernel).

The loop is src/GPU/gpu.cc:52-83 (find_corresponding_opti).  Every search returns the exact fp64
first minimum whichever path runs it (the bundle cascade or the grid), so a registration must
follow the same trajectory bit for bit however the images come to be built and whichever
transform form preceded each search.  Cases:

  * C5 sizes (a 2^20-point shard against the 2^23-point model, BASELINE configs[4]) rotated 30°
    with the images left to their first use (ICP_EAGER_BUNDLE=0, the default since round 5): the
    policy turns to the bundle cascade mid-run and builds the images between two iterations.  Twice on one context
    with icp_set_model in between -- the second registration is the one the round-4 stall hit
    (its transforms wrote global-form slot records for a search that, its images built in
    between, ran the local form) -- against a fresh context with the eager build, bit for bit,
    and 64 queries of the last search against the oracle's brute force over all 2^23 points.
  * a run that ends on slot-record transforms (bundle searches from the first, images built
    before the scene) and a second run carrying over onto the grid: the grid reads the seed
    distances the slot-record transform wrote.
  * the AUTO variant, then the GRID variant on the same context at the slot-order size: the
    grid variant's transforms never write slot records (a write through a null
    seed16 before).
  * ICP_KD_HOST=1 (the host kd order, built inside icp_set_model) with two models of different
    sizes on one context (the build read the previous model's point count).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def registration(ctx, m, p, iters):
    """set_model + set_scene + iters - 1 iterations, a snapshot, one more iteration (whose
    search ran on the snapshot)."""
    ctx.set_model(m)
    ctx.set_scene(p)
    ctx.set_index_digest(iters - 1)
    res, errs = ctx.run(iters - 1, -1.0)
    dig = ctx.index_digest(iters - 1)
    snap = ctx.get_scene()
    res1, errs1 = ctx.run(1, -1.0)
    return dict(errs=np.concatenate([errs, errs1]), dig=dig, snap=snap, idx=ctx.get_indices(),
                scene=ctx.get_scene(), s=res1.s, R=np.array(res1.R[:]), t=np.array(res1.t[:]))


def assert_same(a, b):
    assert np.array_equal(a["errs"], b["errs"])
    assert np.array_equal(a["dig"], b["dig"])
    assert np.array_equal(a["idx"], b["idx"])
    assert np.array_equal(a["scene"], b["scene"])
    assert a["s"] == b["s"] and np.array_equal(a["R"], b["R"]) and np.array_equal(a["t"], b["t"])


def test_c5_shard_mid_run_bundle_build(amd, oracle, monkeypatch):
    n = 1 << 23
    m, p = amd.synthetic_pair(n, seed=42, angle_deg=30.0)  # (far enough that the policy turns to the bundle)
    b, c = amd.shard_range(n, 0, 8)
    shard = np.ascontiguousarray(p[b:b + c])
    iters = 12
    monkeypatch.setenv("ICP_EAGER_BUNDLE", "0")
    with amd.Context(0) as ctx:
        ctx.set_allow_unequal(True)
        reps = []
        for _ in range(2):
            ctx.reset_stats()
            r = registration(ctx, m, shard, iters)
            r["st"] = ctx.stats()
            reps.append(r)
    monkeypatch.setenv("ICP_EAGER_BUNDLE", "1")
    with amd.Context(0) as ctx:
        ctx.set_allow_unequal(True)
        eager = registration(ctx, m, shard, iters)
        est = ctx.stats()
    for r in reps:
        st = r["st"]
        # the images were pending at the run's start and built between two of its iterations,
        # after grid searches and before bundle searches
        assert st["bundle_builds_in_run"] == 1, st
        assert st["run_grid_searches"] >= 1 and st["run_bundle_searches"] >= 1, st
        assert st["grid_fallback"] <= 64, st  # (no flood of queries down to the brute force)
    assert est["bundle_builds_in_run"] == 0 and est["bundle_builds"] == 1, est
    assert_same(reps[0], reps[1])
    assert_same(reps[0], eager)
    # the last search (on the snapshot) against the oracle over all 2^23 model points
    rng = np.random.default_rng(7)
    sel = np.unique(np.concatenate([[0, c - 1], rng.choice(c, 62, replace=False)]))
    _, ref = oracle.closest_blocked(reps[1]["snap"][sel], m)
    assert np.array_equal(reps[1]["idx"][sel], ref)


def test_carry_after_slot_record_transforms(amd):
    """Images built before the scene: the run starts on the bundle cascade and its transforms
    write the slot records (the next search a bundle one); the next run carries over onto the
    grid from the seed distances those transforms wrote."""
    n = 1 << 16
    m, p = amd.synthetic_pair(n, seed=5)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.model_order(n)  # (builds the bundle images: nothing pending at the run's start)
        ctx.set_scene(p)
        ctx.reset_stats()
        ctx.run(2, -1.0)
        st1 = ctx.stats()
        ctx.reset_stats()
        ctx.set_index_digest(10)
        _, errs = ctx.run(10, -1.0)
        a = dict(errs=errs, dig=ctx.index_digest(10), scene=ctx.get_scene(), st=ctx.stats())
    with amd.Context(0) as ctx:  # (the same split: each run's first iteration is the two-pass moments)
        ctx.set_nn_variant(amd.VARIANT_BUNDLE)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(2, -1.0)
        ctx.set_index_digest(10)
        _, errs = ctx.run(10, -1.0)
        b = dict(errs=errs, dig=ctx.index_digest(10), scene=ctx.get_scene())
    assert st1["run_bundle_searches"] == 2, st1
    assert a["st"]["run_grid_searches"] >= 1, a["st"]
    assert np.array_equal(a["dig"], b["dig"])
    assert np.array_equal(a["errs"], b["errs"])
    assert np.array_equal(a["scene"], b["scene"])


def rotation(deg, axis=(1.0, 2.0, 3.0)):
    a = np.asarray(axis) / np.linalg.norm(axis)
    t = np.deg2rad(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def test_auto_then_grid_variant_on_one_context(amd, oracle):
    n = 1 << 16
    rng = np.random.default_rng(11)
    m = rng.uniform(-1, 1, size=(n, 3))
    p = m @ rotation(60.0).T + np.array([0.3, -0.2, 0.1])  # far: the bundle cascade, records sized
    p2 = m @ rotation(4.0).T + np.array([0.02, 0.01, -0.03])
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(6, -1.0)
        assert ctx.stats()["run_bundle_searches"] >= 2
        ctx.set_nn_variant(amd.VARIANT_GRID)
        ctx.set_scene(p2)
        ctx.set_index_digest(6)
        _, errs = ctx.run(5, -1.0)
        snap = ctx.get_scene()
        _, e1 = ctx.run(1, -1.0)
        a = dict(errs=np.concatenate([errs, e1]), idx=ctx.get_indices(), scene=ctx.get_scene())
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(amd.VARIANT_GRID)
        ctx.set_model(m)
        ctx.set_scene(p2)
        _, errs = ctx.run(5, -1.0)
        _, e1 = ctx.run(1, -1.0)
        b = dict(errs=np.concatenate([errs, e1]), idx=ctx.get_indices(), scene=ctx.get_scene())
    assert np.array_equal(a["errs"], b["errs"])
    assert np.array_equal(a["idx"], b["idx"])
    assert np.array_equal(a["scene"], b["scene"])
    sel = np.sort(rng.choice(n, 256, replace=False))
    _, ref = oracle.closest_blocked(snap[sel], m)
    assert np.array_equal(a["idx"][sel], ref)


KD_HOST_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import icp_amd, oracle_py
rng = np.random.default_rng(3)
with icp_amd.Context(0) as ctx:
    ctx.set_nn_variant(icp_amd.VARIANT_BUNDLE)
    for nm in (1 << 14, 3 * (1 << 15) + 517, 1 << 14):
        m = rng.uniform(-1, 1, size=(nm, 3))
        ctx.set_model(m)
        kd = ctx.model_order(nm)
        assert np.array_equal(np.sort(kd), np.arange(nm)), "kd order is not a permutation"
        q = m[rng.choice(nm, 1 << 14, replace=False)] + rng.normal(scale=0.01, size=(1 << 14, 3))
        _, idx = ctx.closest_matrix(q)
        assert ctx.stats()["last_filter"] == 3, ctx.stats()["last_filter"]
        _, ref = oracle_py.closest_blocked(q, m)
        assert np.array_equal(idx, ref), nm
print("kd_host ok")
"""


def test_kd_host_models_of_different_sizes(amd):
    env = dict(os.environ, ICP_KD_HOST="1")
    r = subprocess.run([sys.executable, "-c", KD_HOST_SCRIPT, os.path.join(ROOT, "iterative-closest-point_amd"),
                        os.path.join(ROOT, "oracle")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "kd_host ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("case", ["slot_order", "one_launch"])
def test_progress_callback_streams_each_iteration(amd, case):
    """icp_set_progress (the reference prints each iteration's error as it ends, gpu.cc:65,77):
    one call per recorded iteration, in order, with the trace's values -- on the launch loop
    (a slot-order scene, its errors reported while the run waits) and on the one-launch path."""
    if case == "slot_order":
        m, p = amd.synthetic_pair(1 << 16, seed=9)
        iters, thr = 7, -1.0
    else:
        import datasets
        m = amd.load_matrix(datasets.path("cow_ref"))
        p = amd.load_matrix(datasets.path("cow_tr1"))
        iters, thr = 20, 1e-5
    seen = []
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.set_progress(lambda i, e: seen.append((i, e)))
        res, errs = ctx.run(iters, thr)
        ctx.set_progress(None)
        ctx.run(1, -1.0)  # (off: nothing more)
    assert [i for i, _ in seen] == list(range(res.iterations))
    assert np.array_equal(np.array([e for _, e in seen]), errs)
