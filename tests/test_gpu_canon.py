"""The canonical schedule and the fused grid iteration (icp_canon.h, icp_canon.hip,
icp_grid.hip nn_grid_iter_kernel, icp_engine.hip run_loop).

The loop is src/GPU/gpu.cc:52-83: per iteration the exact NN of every point, the alignment
(gpu.cc:95-151) and the transform with its residual.  Every path that produces an iteration's
sums writes the same canonical rows (32-point chunk trees, strands, rows, one fold), so:

  * the fused kernel (transform + seeded search + moments in one launch, the default) and the
    separate kernels of the same schedule (ICP_GRID_ITER=0) give the same trajectory bit for bit:
    errors, per-iteration index digests, final scene and transform -- on a whole scene, on a
    sparse shard (a W = 8 rank's share against the whole model) and on a scene of two chunks a
    strand (2^20); so does the fused kernel's opt-in four-lane form (ICP_ITER_WIDE=1, scenes of
    at most 2^19 points: two waves a chunk, the chunk's halves joined as the 32-leaf tree's last
    step);
  * the round-4 schedule (ICP_CANON=0: per-path reduction orders) finds the same correspondences
    in every iteration (digests equal) and errors equal to rounding (rtol 1e-12).

Each setting runs in its own process (the switches are read once per process).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import icp_amd
out = {}
iters = 12
for name, n, frac in (("whole", 1 << 17, 1), ("shard", 1 << 19, 8), ("big", 1 << 20, 1)):
    m, p = icp_amd.synthetic_pair(n, seed=31, angle_deg=6.0)
    b, c = icp_amd.shard_range(n, 0, frac)
    scene = np.ascontiguousarray(p[b:b + c])
    with icp_amd.Context(0) as ctx:
        ctx.set_allow_unequal(True)
        ctx.set_model(m)
        ctx.set_scene(scene, np_total=c)
        ctx.set_index_digest(iters)
        res, errs = ctx.run(iters, -1.0)
        out[name + "_errs"] = errs
        out[name + "_dig"] = ctx.index_digest(iters)
        out[name + "_scene"] = ctx.get_scene()
        out[name + "_xf"] = np.concatenate([[res.s], np.array(res.R[:]), np.array(res.t[:])])
        out[name + "_grid"] = np.array([ctx.stats()["run_grid_searches"]])
# a scene 1e3 model spreads away (ADVICE r05: the first iteration's one-pass moments around a shift
# far from the scene cancel (D / sigma)^2 of their precision), and a positive threshold that stops
# the run mid-way (ADVICE r05: the lagged error test of the canonical schedule)
m, p = icp_amd.synthetic_pair(1 << 17, seed=33, angle_deg=6.0)
for name, scene, thr in (("far", p + np.array([1000.0, -700.0, 500.0]), -1.0), ("thresh", p, None)):
    if thr is None:  # (the threshold: between the trajectory's 6th and 7th errors)
        with icp_amd.Context(0) as ctx:
            ctx.set_model(m)
            ctx.set_scene(scene)
            _, e = ctx.run(12, -1.0)
        thr = float(0.5 * (e[5] + e[6]))
        out["thresh_full_errs"] = e
    with icp_amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(scene)
        res, errs = ctx.run(12 if name == "thresh" else 6, thr)
        out[name + "_errs"] = errs
        out[name + "_iters"] = np.array([res.iterations, res.converged])
        out[name + "_scene"] = ctx.get_scene()
        out[name + "_xf"] = np.concatenate([[res.s], np.array(res.R[:]), np.array(res.t[:])])
np.savez(sys.argv[2], **out)
print("canon ok")
"""


def run_setting(tmp_path, name, env):
    out = str(tmp_path / f"canon_{name}.npz")
    r = subprocess.run([sys.executable, "-c", SCRIPT, os.path.join(ROOT, "iterative-closest-point_amd"), out],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
    assert r.returncode == 0 and "canon ok" in r.stdout, r.stdout + r.stderr
    return dict(np.load(out))


@pytest.fixture(scope="module")
def settings(icp_lib, tmp_path_factory):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    tmp = tmp_path_factory.mktemp("canon")
    return {"fused": run_setting(tmp, "fused", {}),
            "wide": run_setting(tmp, "wide", {"ICP_ITER_WIDE": "1"}),
            "separate": run_setting(tmp, "separate", {"ICP_GRID_ITER": "0"}),
            "round4": run_setting(tmp, "round4", {"ICP_CANON": "0"})}


@pytest.mark.parametrize("other", ["separate", "wide"])
@pytest.mark.parametrize("case", ["whole", "shard", "big"])
def test_fused_equals_separate_bitwise(settings, case, other):
    a, b = settings["fused"], settings[other]
    assert a[case + "_grid"][0] >= 8  # (the grid's seeded iterations ran: the fused kernel's path)
    for k in ("errs", "dig", "scene", "xf"):
        assert np.array_equal(a[f"{case}_{k}"], b[f"{case}_{k}"]), k


@pytest.mark.parametrize("case", ["whole", "shard", "big"])
def test_canonical_matches_round4_schedule(settings, case):
    a, b = settings["fused"], settings["round4"]
    assert np.array_equal(a[case + "_dig"], b[case + "_dig"])
    np.testing.assert_allclose(a[case + "_errs"], b[case + "_errs"], rtol=1e-12)
    np.testing.assert_allclose(a[case + "_scene"], b[case + "_scene"], rtol=0, atol=1e-12)


def test_far_scene_first_iteration_matches_two_pass(settings):
    """A scene 1e3 spreads from the model: the canonical first iteration sums its moments around the
    scene's own centroid (all ranks' sum, icp_engine.hip run_loop), so its (s, R, t) agree with the
    reference's two passes (gpu.cc:98-104, the round-4 schedule) to rounding."""
    a, b = settings["fused"], settings["round4"]
    np.testing.assert_allclose(a["far_errs"], b["far_errs"], rtol=1e-12)
    np.testing.assert_allclose(a["far_xf"], b["far_xf"], rtol=1e-12, atol=1e-12)
    ext = float(np.abs(b["far_scene"]).max())
    np.testing.assert_allclose(a["far_scene"], b["far_scene"], rtol=0, atol=1e-12 * ext)


def test_threshold_stops_where_the_reference_breaks(settings):
    """A positive threshold on a slot-order scene (2^17): the run stops after the first iteration whose
    err is below it (gpu.cc:79-80) -- the lagged error test of the canonical schedule freezes the
    scene at the same point -- with the round-4 schedule's iteration count, errors (rtol 1e-12),
    scene and transform."""
    a, b = settings["fused"], settings["round4"]
    full = a["thresh_full_errs"]
    thr = 0.5 * (full[5] + full[6])
    want = int(np.argmax(full < thr)) + 1
    assert a["thresh_iters"][0] == b["thresh_iters"][0] == want
    assert a["thresh_iters"][1] == b["thresh_iters"][1] == 1
    np.testing.assert_allclose(a["thresh_errs"], b["thresh_errs"], rtol=1e-12)
    np.testing.assert_allclose(a["thresh_errs"], full[:want], rtol=0)
    np.testing.assert_allclose(a["thresh_scene"], b["thresh_scene"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(a["thresh_xf"], b["thresh_xf"], rtol=1e-12, atol=1e-12)
