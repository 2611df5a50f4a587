"""Adversarial scenes for the f16 MFMA filter's certificate (nn_finalize_mfma16_kernel).

The default NN path's exactness rests on the certificate's error envelope, which is derived
from the measured accumulation behaviour of v_mfma_f32_32x32x16_f16.  These
scenes sit on the envelope's worst cases; on each, at >= 2^18 queries, the f16 path (unseeded
closest_matrix and the seeded searches of icp_run) must return exactly the fp64 brute force's
indices (the reference's first-minimum rule), and the certificate audit (icp_set_cert_audit)
must show the winner's filter error below its bound on every certified query:

  near_ties     queries equidistant (to within rounding) from 2-8 model points
  top_of_range  scaled coordinates at the top of [2^11, 2^12) (largest hi/lo products)
  subnormal_lo  model coordinates whose f16 lo halves are subnormal (aligned as 2^-14)
  far_queries   queries with |a_s| just inside the clamp kF16QueryClamp = 32000
  clusters      a 1e6-extent model of tight 1e-3 clusters (relative near ties): below the f16
                resolution at that scale, so the certificate must refuse every query (all of
                them go to the exact grid level)

The audit's two figures (max |G^ - G64| / delta_b, min certified margin) are printed and
written to gpurun_out/cert_stress.json when that directory exists; DESIGN.md §3.1 quotes them.
Behind the bundle bound, icp_bundle_audit also checks its exclusions on every scene: the MFMA's
bound value against its folded margins, and the geometry of the excluded bundles near the bound.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NQ = 1 << 18
CLAMP = 32000.0


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def unit_vectors(rng, k):
    v = rng.normal(size=(k, 3))
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def scene_near_ties(rng):
    # 2^15 centres, each with 2-8 model points at the same fp64 distance r (up to rounding),
    # over a background of uniform points; queries = the centres + jittered copies
    nc = 1 << 15
    centres = rng.uniform(-1, 1, size=(nc, 3))
    pts = []
    for c in centres:
        k = rng.integers(2, 9)
        r = rng.uniform(0.002, 0.02)
        pts.append(c + r * unit_vectors(rng, k))
    m = np.concatenate(pts + [rng.uniform(-1, 1, size=(1 << 17, 3))])
    m = m[rng.permutation(m.shape[0])]
    q = np.concatenate([centres, centres + rng.normal(scale=1e-9, size=centres.shape),
                        rng.uniform(-1, 1, size=(NQ - 2 * nc, 3))])
    return m, q


def scene_top_of_range(rng):
    # centroid exactly 0 (symmetric model) and max |m| = 4095.75: scale 2^0, scaled coordinates
    # up to the top of [2^11, 2^12)
    h = rng.uniform(-4095.75, 4095.75, size=(1 << 17, 3))
    h[0] = [4095.75, -4095.75, 4095.75]
    m = np.concatenate([h, -h])
    q = m[rng.integers(0, m.shape[0], NQ)] + rng.normal(scale=0.5, size=(NQ, 3))
    return m, q


def scene_subnormal_lo(rng):
    # scale 1, centroid 0: x = k + j 2^-20 with k even (exact f16 hi) and j in 1..7, so that
    # lo = j 2^-20 < 2^-14 is an f16 subnormal; queries on the same lattice (exact ties)
    n = 1 << 17
    k = rng.integers(-2047, 2048, size=(n, 3)) * 2.0
    j = rng.integers(1, 8, size=(n, 3)) * 2.0 ** -20
    h = k + j
    h[0] = [4094.0 + 2.0 ** -20] * 3
    m = np.concatenate([h, -h])
    q = m[rng.integers(0, m.shape[0], NQ)] + rng.integers(-3, 4, size=(NQ, 3)) * 2.0 ** -19
    return m, q


def scene_far_queries(rng):
    # model in [-1, 1]^3 (max |m - c| ~ 1 -> scale 2^11), queries at |a_s| in (31500, 32000):
    # far outside the model, near the clamp beyond which queries are never certified
    m = rng.uniform(-1, 1, size=(1 << 18, 3))
    c = m.mean(axis=0)
    rm = np.abs(m - c).max()
    scale = 2.0 ** np.floor(np.log2(4096.0 / rm))
    while rm * scale >= 4096.0:
        scale *= 0.5
    d = unit_vectors(rng, NQ)
    d /= np.abs(d).max(axis=1, keepdims=True)  # max-norm 1: |a_s| per axis = the radius
    rad = rng.uniform(31500.0, 31999.0, size=(NQ, 1)) / scale
    return m, c + d * rad


def scene_clusters(rng):
    # 2^11 clusters of 128 points within 1e-3, spread over a 1e6 extent
    nc = 1 << 11
    centres = rng.uniform(-5e5, 5e5, size=(nc, 3))
    m = (centres[:, None, :] + rng.normal(scale=1e-3, size=(nc, 128, 3))).reshape(-1, 3)
    q = m[rng.integers(0, m.shape[0], NQ)] + rng.normal(scale=5e-4, size=(NQ, 3))
    return m, q


SCENES = {"near_ties": scene_near_ties, "top_of_range": scene_top_of_range,
          "subnormal_lo": scene_subnormal_lo, "far_queries": scene_far_queries,
          "clusters": scene_clusters}
AUDIT = {}


def run(amd, nn_mode, variant, m, q, iters):
    with amd.Context(0, nn_mode) as ctx:
        ctx.set_nn_variant(variant)
        ctx.set_allow_unequal(m.shape[0] != q.shape[0])
        ctx.set_model(m)
        if nn_mode == amd.NN_CERTIFIED:
            ctx.set_cert_audit(True)
        _, idx0 = ctx.closest_matrix(q)
        st0 = ctx.stats()
        ctx.reset_stats()
        ctx.set_scene(q)
        res, errs = ctx.run(iters, -1.0)
        # the bundle bound's exclusions audited against the last correspondences as seeds
        audit = ctx.bundle_audit(64) if variant == amd.VARIANT_BUNDLE else None
        return idx0, st0, res, errs, ctx.get_scene(), ctx.get_indices(), ctx.stats(), audit


@pytest.mark.parametrize("variant", ["mfma16", "bundle"])
@pytest.mark.parametrize("name", list(SCENES))
def test_f16_certificate_adversarial(amd, name, variant):
    """The f16 certificate on its worst cases, behind the full N x M filter and behind the
    bundle bound (whose exclusions must never drop the answer or a tie of it)."""
    rng = np.random.default_rng(list(SCENES).index(name) + 101)
    m, q = SCENES[name](rng)
    assert q.shape[0] >= NQ
    d = run(amd, amd.NN_CERTIFIED, amd.VARIANT_MFMA16 if variant == "mfma16" else amd.VARIANT_BUNDLE, m, q, 3)
    f = run(amd, amd.NN_FP64, 0, m, q, 3)
    # unseeded search: identical indices
    np.testing.assert_array_equal(d[0], f[0])
    # three icp_run iterations (the second and third seeded): bitwise the same run
    assert d[2].iterations == f[2].iterations == 3
    np.testing.assert_array_equal(d[3], f[3])
    np.testing.assert_array_equal(d[4], f[4])
    np.testing.assert_array_equal(d[5], f[5])
    for st, searched in ((d[1], NQ), (d[6], 3 * q.shape[0])):
        # every query of every search is either certified (and audited) or queued to the exact
        # levels; a scene whose near ties lie below the f16 resolution certifies nothing
        assert st["cert_audited"] + st["level1_queued"] == searched, st
        if st["cert_audited"]:
            assert st["cert_max_err_ratio"] < 1.0, st  # the bound held on every certified winner
    if name != "clusters":
        assert d[1]["cert_audited"] > 0 and d[6]["cert_audited"] > 0
    if variant != "mfma16":
        #  the bundle exclusions keep their margin: the MFMA's V^ off the value its
        # operands represent by less than the folded margins mu_q + mu_c on every evaluated
        # (query, bundle) pair, and no excluded bundle near the bound holds a point as close as
        # the seed
        au = d[7]
        print(name, "bundle audit", json.dumps(au))
        assert au["violations"] == 0, au
        if au["pairs"]:
            assert au["max_err_ratio"] < 1.0, au
        if name not in ("clusters", "far_queries"):
            assert au["pairs"] > 0 and au["checked"] > 0, au
        AUDIT.setdefault("bundle_audit", {})[name] = au
        _dump()
        return
    AUDIT[name] = {"unseeded": {k: d[1][k] for k in ("cert_max_err_ratio", "cert_min_margin", "cert_audited",
                                                     "level1_queued", "grid_fallback")},
                   "icp_run": {k: d[6][k] for k in ("cert_max_err_ratio", "cert_min_margin", "cert_audited",
                                                    "level1_queued", "grid_fallback")},
                   "n_model": int(m.shape[0]), "n_queries": int(q.shape[0])}
    print(name, json.dumps(AUDIT[name]))
    _dump()


def _dump():
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "cert_stress.json"), "w") as fh:
            json.dump(AUDIT, fh, indent=1)
