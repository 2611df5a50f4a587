"""The bench's own workloads, parity-checked (BASELINE.json configs C4 and C5).

C4 (bench.py's timed workload): the 2^20-point synthetic pair, 30 fixed iterations, run
through icp_run exactly as bench.py runs it, in the default path (f16 MFMA filter +
certificate + grid resolver), in ICP_NN_FP64 and in the grid variant.  The three runs must be
bitwise identical (same correspondences => same arithmetic), and must match the oracle's
trajectory (tests/golden/c4_oracle.json, made by tests/golden/make_c4.py from the C
restatement of src/cpu.cc:55-79):
  * per-iteration correspondence digests (sum idx, sum (j+1) idx[j], #identity): exact;
  * per-iteration err: rel 1e-9; last (s, R, t): abs 1e-9; final cloud: abs 1e-9 on the
    sampled rows and rel 1e-9 on the per-axis sums (fp64 throughout; the reduction order is
    the only difference from the oracle).

C5 (2^23-point pair, 8 GPUs): the rank-0 shard of the scene (2^20 queries) against the full
2^23-point model, on one GPU: two iterations, then a third whose search is seeded from the
second's correspondences (the kernel every C5 rank runs from iteration 2 on).  Default and
ICP_NN_FP64 must agree bitwise (errors, scene, indices); a sample of the third search's
queries is checked against the oracle's brute force over all 2^23 model points.
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
C4_FIXTURE = os.path.join(HERE, "golden", "c4_oracle.json")


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_c4(amd, m, p, nn_mode, variant, iters):
    with amd.Context(0, nn_mode) as ctx:
        ctx.set_nn_variant(variant)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.set_index_digest(iters)
        res, errs = ctx.run(iters, -1.0)  # bench.py: fixed iterations, threshold disabled
        dig = ctx.index_digest(iters)
        out = ctx.get_scene()
        st = ctx.stats()
    return res, errs, dig, out, st


def test_c4_trajectory_matches_oracle(amd):
    with open(C4_FIXTURE) as f:
        fx = json.load(f)
    n, iters = fx["n"], fx["iters"]
    m, p = amd.synthetic_pair(n, seed=fx["seed"])
    assert sha(m) == fx["model_sha256"] and sha(p) == fx["scene_sha256"]

    runs = {"default": run_c4(amd, m, p, amd.NN_CERTIFIED, amd.VARIANT_AUTO, iters),
            "fp64": run_c4(amd, m, p, amd.NN_FP64, amd.VARIANT_AUTO, iters),
            "grid": run_c4(amd, m, p, amd.NN_CERTIFIED, amd.VARIANT_GRID, iters),
            "bundle": run_c4(amd, m, p, amd.NN_CERTIFIED, amd.VARIANT_BUNDLE, iters),
            "mfma16": run_c4(amd, m, p, amd.NN_CERTIFIED, amd.VARIANT_MFMA16, iters)}
    res, errs, dig, out, st = runs["default"]
    assert res.iterations == iters
    # the default path is the f16 MFMA filter and its certificate sent queries onward
    assert st["level1_queued"] > 0
    for name in ("fp64", "grid", "bundle", "mfma16"):
        r2, e2, d2, o2, _ = runs[name]
        assert np.array_equal(e2, errs), name
        assert np.array_equal(d2, dig), name
        assert np.array_equal(o2, out), name
        assert (r2.s, list(r2.R), list(r2.t)) == (res.s, list(res.R), list(res.t)), name

    for k in range(iters):
        want = fx["idx"][k]
        got = [int(x) for x in dig[k]]
        assert got == [want["sum"], want["wsum"], want["identity"]], f"iteration {k} correspondences differ"
    np.testing.assert_allclose(errs, fx["err"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(res.s, fx["s"][-1], rtol=0, atol=1e-9)
    np.testing.assert_allclose(np.array(res.R), np.array(fx["R"][-1]), rtol=0, atol=1e-9)
    np.testing.assert_allclose(np.array(res.t), np.array(fx["t"][-1]), rtol=0, atol=1e-9)
    rows = np.array(fx["final"]["rows"])
    np.testing.assert_allclose(out[rows], np.array(fx["final"]["sample"]), rtol=0, atol=1e-9)
    np.testing.assert_allclose(out.sum(axis=0), fx["final"]["sum"], rtol=1e-9, atol=1e-9)


def test_c5_rank0_shard(amd, oracle):
    n = 1 << 23
    m, p = amd.synthetic_pair(n, seed=42)
    b, c = amd.shard_range(n, 0, 8)
    shard = np.ascontiguousarray(p[b:b + c])
    assert c == 1 << 20

    def run(nn_mode):
        with amd.Context(0, nn_mode) as ctx:
            ctx.set_allow_unequal(True)  # one shard against the whole model
            ctx.set_model(m)
            ctx.set_scene(shard)
            _, e1 = ctx.run(2, -1.0)
            s2 = ctx.get_scene()
            _, e2 = ctx.run(1, -1.0)  # seeded from the second iteration's correspondences
            idx3 = ctx.get_indices()
            s3 = ctx.get_scene()
            st = ctx.stats()
        return np.concatenate([e1, e2]), s2, idx3, s3, st

    e_d, s2_d, idx_d, s3_d, st = run(amd.NN_CERTIFIED)
    e_f, s2_f, idx_f, s3_f, _ = run(amd.NN_FP64)
    assert st["level1_queued"] > 0  # the f16 filter ran and queued near ties onward
    assert np.array_equal(idx_d, idx_f)
    assert np.array_equal(e_d, e_f)
    assert np.array_equal(s2_d, s2_f) and np.array_equal(s3_d, s3_f)
    assert idx_d.min() >= 0 and idx_d.max() < n
    # the oracle's brute force over all 2^23 model points, on a sample of the third search
    rng = np.random.default_rng(5)
    sel = np.sort(np.concatenate([rng.choice(c, 192, replace=False), [0, c - 1]]))
    _, ref = oracle.closest_blocked(s2_d[sel], m)
    assert np.array_equal(idx_d[sel], ref)
