"""icp_set_model's preparation on the device (icp_model.hip).

* The bundle filter's kd order: every 32-point bundle (and every 1,024-point block) holds
  exactly the points of the host rule (icp_bundle.hip bundle_kd_order: a range of more than
  1,024 points splits at a multiple of 1,024, one of more than 32 at a multiple of 32, at
  ceil(units / 2) units along the widest axis of its box, points ordered by (coordinate,
  original index)).  Checked against a recursive statement of the rule (small clouds with many
  exact ties) and a level-by-level numpy statement (C4 size, ragged sizes).
* The device checks of the model: non-finite coordinates and fp32 overflow are refused with
  ICP_E_RANGE, and a refused model leaves no half-built state behind.
* icp_ensure_model on a model too large for the host copy: an exact device comparison
  (no hash), so a one-ulp change is always a new model.
"""
import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(7)


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def kd_sets_recursive(m):
    """bundle_kd_order's rule, recursively (pure Python; small clouds)."""
    order = list(range(m.shape[0]))

    def split(lo, hi):
        cnt = hi - lo
        unit = 1024 if cnt > 1024 else 32 if cnt > 32 else 0
        if not unit:
            return
        pts = m[order[lo:hi]]
        ext = pts.max(axis=0) - pts.min(axis=0)
        ax = 0
        for a in (1, 2):
            if ext[a] > ext[ax]:
                ax = a
        units = (cnt + unit - 1) // unit
        mid = lo + unit * ((units + 1) // 2)
        order[lo:hi] = sorted(order[lo:hi], key=lambda j: (m[j, ax], j))
        split(lo, mid)
        split(mid, hi)

    split(0, m.shape[0])
    return np.array(order)


def kd_sets_levels(m):
    """The same rule level by level in numpy (every range of a level at once; C4 size)."""
    n = m.shape[0]
    perm = np.arange(n)
    lo = np.array([0]); hi = np.array([n])
    while True:
        cnt = hi - lo
        unit = np.where(cnt > 1024, 1024, np.where(cnt > 32, 32, 0))
        act = unit > 0
        if not act.any():
            return perm
        units = np.where(act, (cnt + np.maximum(unit, 1) - 1) // np.maximum(unit, 1), 0)
        mid = lo + unit * ((units + 1) // 2)
        pts = m[perm]
        ext = np.maximum.reduceat(pts, lo, axis=0) - np.minimum.reduceat(pts, lo, axis=0)
        ax = np.zeros(lo.size, dtype=int)
        for a in (1, 2):
            ax = np.where(ext[:, a] > ext[np.arange(lo.size), ax], a, ax)
        seg = np.repeat(np.arange(lo.size), cnt)
        pos = np.arange(n)
        # sort key within a range: its axis coordinate (active), else its position (kept)
        sec = np.where(act[seg], pts[pos, ax[seg]], (pos - lo[seg]).astype(np.float64))
        perm = perm[np.lexsort((perm, sec, seg))]
        nlo = np.concatenate([np.stack([lo[act], mid[act]], 1).ravel(), lo[~act]])
        nhi = np.concatenate([np.stack([mid[act], hi[act]], 1).ravel(), hi[~act]])
        o = np.argsort(nlo, kind="stable")
        lo, hi = nlo[o], nhi[o]


def bundle_sets(order):
    n = order.size
    nb = (n + 31) // 32
    return [frozenset(order[32 * b:min(n, 32 * b + 32)].tolist()) for b in range(nb)]


@pytest.mark.parametrize("n,quant", [(8192, None), (20000, 0.125), (33000, 1.0 / 64), (12345, None)])
def test_kd_order_matches_host_rule_small(amd, n, quant):
    m = RNG.uniform(-1, 1, size=(n, 3))
    if quant:  # many exact coordinate ties: the (coordinate, index) order decides
        m = np.round(m / quant) * quant
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        kd = ctx.model_order(n)
    assert np.array_equal(np.sort(kd), np.arange(n))
    assert bundle_sets(kd) == bundle_sets(kd_sets_recursive(m))


@pytest.mark.parametrize("n", [1 << 20, 1048576 + 777])
def test_kd_order_matches_host_rule_c4(amd, n):
    m, _ = amd.synthetic_pair(n, seed=42) if n == 1 << 20 else (RNG.normal(size=(n, 3)), None)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        kd = ctx.model_order(n)
    ref = kd_sets_levels(m)
    assert bundle_sets(kd) == bundle_sets(ref)
    # and the 1,024-point blocks
    nb = (n + 1023) // 1024
    assert all(set(kd[1024 * b:1024 * b + 1024].tolist()) == set(ref[1024 * b:1024 * b + 1024].tolist())
               for b in range(nb))


def test_kd_order_surface_cloud(amd):
    """horse_ref (a surface cloud, 48,485 points): the rule on real data."""
    m = amd.load_matrix(datasets.path("horse_ref"))
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        kd = ctx.model_order(m.shape[0])
    assert bundle_sets(kd) == bundle_sets(kd_sets_levels(m))


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf, 1e300])
def test_model_checks_refuse_and_leave_no_state(amd, bad):
    good = RNG.normal(size=(9000, 3))
    m = good.copy()
    m[4321, 1] = bad
    p = good[:500] + 0.01
    with amd.Context(0) as ctx:
        with pytest.raises(amd.ICPError) as e:
            ctx.set_model(m)
        assert e.value.code == amd.ICP_E_RANGE
        with pytest.raises(amd.ICPError):
            ctx.closest_matrix(p)  # no model: refused, not answered from a half-built one
        ctx.set_model(good)
        _, idx = ctx.closest_matrix(p)
    d = ((p[:, None, :] - good[None, :, :]) ** 2).sum(-1)
    assert np.array_equal(idx, d.argmin(axis=1))


def test_ensure_model_large_is_exact(amd):
    """70,000 points: no host copy, so the comparison runs on the device, bit for bit."""
    m = RNG.uniform(-1, 1, size=(70000, 3))
    p = m[:3000] + RNG.normal(scale=1e-3, size=(3000, 3))
    with amd.Context(0) as ctx:
        assert ctx.ensure_model(m) is True
        assert ctx.ensure_model(m.copy()) is False
        _, i1 = ctx.closest_matrix(p)
        m2 = m.copy()
        m2[i1[0]] = np.nextafter(m2[i1[0]], 10.0)  # one ulp on one point
        assert ctx.ensure_model(m2) is True
        assert ctx.ensure_model(m2) is False
        m3 = m.copy()
        m3[i1[0]] += 5.0  # move the first query's neighbour away: the answers follow
        assert ctx.ensure_model(m3) is True
        _, i3 = ctx.closest_matrix(p[:1])
        assert i3[0] != i1[0]


@pytest.mark.parametrize("bad", [np.nan, 1e300])
def test_refused_model_keeps_the_resident_one(amd, bad):
    """The model's SoA copy and double4 rows are built into spare buffers while its checks are
    read back (set_model_staged): a refused model must leave the resident model whole -- large
    enough for the device path (no host copy) and searched on the grid after the refusal."""
    rng = np.random.default_rng(3)
    good = rng.uniform(-1.0, 1.0, size=(1 << 17, 3))
    m = rng.uniform(-1.0, 1.0, size=(1 << 17, 3))
    m[777, 2] = bad
    p = good[:4096] + 0.003
    with amd.Context(0) as ctx:
        ctx.set_model(good)
        _, before = ctx.closest_matrix(p)
        with pytest.raises(amd.ICPError) as e:
            ctx.set_model(m)
        assert e.value.code == amd.ICP_E_RANGE
        _, after = ctx.closest_matrix(p)
    assert np.array_equal(before, after)
    sel = np.arange(0, 4096, 64)
    d = ((p[sel, None, :] - good[None, :, :]) ** 2).sum(-1)
    assert np.array_equal(after[sel], d.argmin(axis=1))
