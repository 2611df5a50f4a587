"""icp_run's search policy at the bundle filter's sizes (icp_engine.hip run_loop) and the seeded
grid search it switches to (grid_seeded_search: the per-query walk of boxes up to 125 cells, a
whole wave per query for bigger ones, fp64 brute force over the cell budget).

With the AUTO variant and the scene in slot order, a seeded search takes the grid when the last
transform the host has seen left few points far from their correspondence, else the bundle
cascade.  Both return the exact first minimum, so:
  * the AUTO run's per-iteration index digests equal the explicit bundle variant's (which never
    takes the grid) at every iteration, and its final cloud is bit-identical;
  * the policy engages on a well-aligned pair (last_filter == grid) and stays on the bundle
    cascade while the scene is far from the model;
  * the second pass (big boxes) gives the same answers: clustered clouds (many points a cell)
    and a sparse shard, against the oracle.
Sizes: 2^16 x 2^16 (>= 2^31 pairs, > 49,152 queries: the slot-order path).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1 << 16


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def run(amd, m, p, iters, variant, digest=True):
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(variant)
        ctx.set_model(m)
        ctx.set_scene(p)
        if digest:
            ctx.set_index_digest(iters)
        res, errs = ctx.run(iters, -1.0)
        out = dict(errs=errs, res=res, scene=ctx.get_scene(), idx=ctx.get_indices(), stats=ctx.stats())
        if digest:
            out["dig"] = ctx.index_digest(iters)
    return out


def rotation(deg, axis=(1.0, 2.0, 3.0)):
    a = np.asarray(axis) / np.linalg.norm(axis)
    t = np.deg2rad(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def test_policy_engages_and_matches_bundle(amd):
    m, p = amd.synthetic_pair(N, seed=42)
    a = run(amd, m, p, 20, amd.VARIANT_AUTO)
    b = run(amd, m, p, 20, amd.VARIANT_BUNDLE)
    assert amd.FILTER_NAMES[a["stats"]["last_filter"]] == "grid"  # the tiles ran the last searches
    assert amd.FILTER_NAMES[b["stats"]["last_filter"]] == "bundle"
    assert np.array_equal(a["dig"], b["dig"])
    assert np.array_equal(a["errs"], b["errs"])
    assert np.array_equal(a["scene"], b["scene"])


def test_policy_stays_on_bundle_far_from_the_model(amd):
    """A 60-degree rotation: the first iterations move points by many grid cells."""
    rng = np.random.default_rng(3)
    m = rng.uniform(-1, 1, size=(N, 3))
    p = m @ rotation(60.0).T + np.array([0.3, -0.2, 0.1])
    a = run(amd, m, p, 4, amd.VARIANT_AUTO)
    b = run(amd, m, p, 4, amd.VARIANT_BUNDLE)
    assert amd.FILTER_NAMES[a["stats"]["last_filter"]] == "bundle"
    assert np.array_equal(a["dig"], b["dig"])
    assert np.array_equal(a["scene"], b["scene"])


@pytest.mark.parametrize("trim", ["0", "1"])
@pytest.mark.parametrize("case", ["clustered", "shard"])
def test_seeded_grid_against_oracle(amd, oracle, case, trim, monkeypatch):
    """Dense clusters (hundreds of points a cell region: big boxes for the second pass) and an
    8-way shard's sparse queries; the grid variant's seeded searches against the oracle, with
    the whole box and with its rows trimmed to the seed's sphere (ICP_GRID_TRIM)."""
    monkeypatch.setenv("ICP_GRID_TRIM", trim)
    rng = np.random.default_rng(5)
    if case == "clustered":
        centres = rng.uniform(-1, 1, size=(64, 3))
        m = centres[rng.integers(0, 64, N)] + rng.normal(scale=0.01, size=(N, 3))
        p = m @ rotation(1.0).T + 0.002
        scene = p
        total = N
    else:
        m = rng.uniform(-1, 1, size=(N * 8, 3))
        p = m @ rotation(1.0).T + 0.001
        scene = p[:N]  # (queries at an eighth of the model's density: an 8-way shard's)
        total = N
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(amd.VARIANT_GRID)
        ctx.set_allow_unequal(True)
        ctx.set_model(m)
        ctx.set_scene(scene, np_total=total)
        ctx.run(3, -1.0)  # the last two searches seeded
        got = ctx.get_indices()
        cur = ctx.get_scene()
        ctx.run(1, -1.0)  # one more seeded search, on `cur`
        got2 = ctx.get_indices()
        st = ctx.stats()
    sel = np.sort(rng.choice(scene.shape[0], 512, replace=False))
    _, ref = oracle.closest_blocked(cur[sel], m)
    assert np.array_equal(got2[sel], ref)
    assert got.min() >= 0 and got.max() < m.shape[0]
    assert st["level1_queued"] >= 0


def test_policy_carries_over_to_the_next_run(amd):
    """A run that continues the last one on the same scene starts from that run's far count and
    seed distances (grid searches from its first iteration): the same trajectory as the bundle
    cascade's, and a fresh scene starts over."""
    m, p = amd.synthetic_pair(N, seed=42)
    out = {}
    for name, variant in (("auto", amd.VARIANT_AUTO), ("bundle", amd.VARIANT_BUNDLE)):
        with amd.Context(0) as ctx:
            ctx.set_nn_variant(variant)
            ctx.set_model(m)
            ctx.set_scene(p)
            ctx.run(12, -1.0)
            ctx.reset_stats()
            ctx.set_index_digest(6)
            res, errs = ctx.run(6, -1.0)
            out[name] = dict(errs=errs, dig=ctx.index_digest(6), scene=ctx.get_scene(), st=ctx.stats())
    a, b = out["auto"], out["bundle"]
    assert amd.FILTER_NAMES[a["st"]["last_filter"]] == "grid"
    assert np.array_equal(a["dig"], b["dig"])
    assert np.array_equal(a["errs"], b["errs"])
    assert np.array_equal(a["scene"], b["scene"])


@pytest.mark.parametrize("form,trim", [("f4,2,2", "0"), ("f2,2,2", "0"), ("2,2,2", "0"), ("4,1,2", "0"),
                                       ("2,2,2", "1"), ("f4,2,2", "1"), ("4,2,2", "1")])
def test_seeded_forms_match_bundle(amd, form, trim, monkeypatch):
    """Every instantiated form of the seeded grid kernel (ICP_GRID_SEEDED, read at each launch),
    the fp32-image forms included, with and without the rows trimmed to the seed's sphere
    (ICP_GRID_TRIM, trim_row), returns the bundle cascade's indices bit for bit over a run."""
    monkeypatch.setenv("ICP_GRID_SEEDED", form)
    monkeypatch.setenv("ICP_GRID_TRIM", trim)
    m, p = amd.synthetic_pair(N, seed=42)
    a = run(amd, m, p, 16, amd.VARIANT_AUTO)
    monkeypatch.delenv("ICP_GRID_SEEDED")
    monkeypatch.delenv("ICP_GRID_TRIM")
    b = run(amd, m, p, 16, amd.VARIANT_BUNDLE)
    assert amd.FILTER_NAMES[a["stats"]["last_filter"]] == "grid"
    assert np.array_equal(a["dig"], b["dig"])
    assert np.array_equal(a["scene"], b["scene"])
