"""The per-operation drop-in boundary (src/GPU/gpu.hh:110-116) exactly as the reference calls it.

* icp_subtract_col == substract_col_w (compute.cu:381-416): M - m for ANY caller-given m,
  bitwise (one fp64 subtraction per coordinate), on the mapped small-cloud path and the
  staged large-cloud path.
* icp_ensure_model: the shim's model upload (compute_Y_w_opti re-sends the model each call,
  compute.cu:160) cannot go stale: equal contents at a new address -> no upload; the same
  address refilled with a different cloud -> upload, and the answers follow the new cloud.
* icp-capi-replay (tests/capi_replay.cpp): GPU::ICP::find_corresponding_opti +
  find_alignment (gpu.cc:52-151) replayed call for call through the C ABI -- host means,
  two substract_col_w, host S, y_p_norm_w, Horn, compute_err_w(in_place=false), then
  compute_err_w in place -- against the oracle's trajectory (rel 1e-9) and icp_run.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "iterative-closest-point_amd", "build", "icp-capi-replay")
RNG = np.random.default_rng(2024)


@pytest.fixture(scope="module")
def ctx(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    with icp_lib.Context(0) as c:
        yield c


@pytest.mark.parametrize("n", [1, 4, 2903, 65536, 65537, 300001])
def test_subtract_col_any_vector_bitwise(ctx, n):
    M = RNG.normal(size=(n, 3)) * 10.0 ** RNG.integers(-3, 4, size=(n, 1))
    for m in (M.mean(axis=0), np.array([1.5, -2.25e-3, 7e5]), np.array([np.pi, 0.0, -np.e])):
        out = ctx.subtract_col(M, m)
        assert np.array_equal(out, M - m)  # the same IEEE subtraction, bit for bit


def test_subtract_col_empty_and_errors(icp_lib, ctx):
    out = ctx.subtract_col(np.zeros((0, 3)), [1.0, 2.0, 3.0])
    assert out.shape == (0, 3)


def test_ensure_model_cannot_go_stale(icp_lib, ctx):
    m1 = icp_lib.load_matrix(datasets.path("cow_ref"))
    p = icp_lib.load_matrix(datasets.path("cow_tr1"))
    assert ctx.ensure_model(m1) is True
    assert ctx.ensure_model(m1.copy()) is False  # same contents, new address: no upload
    _, i1 = ctx.closest_matrix(p)
    buf = m1.copy()
    assert ctx.ensure_model(buf) is False
    buf[:] = buf[::-1]  # refill the SAME array with a different cloud (reversed order)
    assert ctx.ensure_model(buf) is True
    _, i2 = ctx.closest_matrix(p)
    n = m1.shape[0]
    # a point's NN in the reversed cloud is the mirrored index (ties aside: cow has none)
    assert np.array_equal(i2, n - 1 - i1)
    buf[7, 1] += 1e-9  # a one-ULP-scale change is still a different model
    assert ctx.ensure_model(buf) is True


@pytest.mark.parametrize("cfg", [("cow_ref", "cow_tr1", "cow_tr1", 20), ("cow_ref", "cow_tr2", "cow_tr2", 20),
                                 ("horse_ref", "horse_tr2", "horse_tr2", 20)])
def test_reference_call_sequence_replay(icp_lib, golden, cfg):
    mname, pname, gname, iters = cfg
    r = subprocess.run([REPLAY, datasets.path(mname), datasets.path(pname), str(iters)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    g = golden[gname]
    assert out["iterations"] == g["iterations"]
    assert out["model_uploads"] == 1  # the model is sent every iteration, uploaded once
    np.testing.assert_allclose(out["err"], g["err"], rtol=1e-9)
    for k, st in enumerate(out["steps"]):
        np.testing.assert_allclose(st["s"], g["s"][k], rtol=0, atol=1e-9)
        np.testing.assert_allclose(np.array(st["R"]).reshape(3, 3), np.array(g["R"][k]), rtol=0, atol=1e-9)
        np.testing.assert_allclose(st["t"], g["t"][k], rtol=0, atol=1e-9)
    # the device-resident loop reaches the same place
    m = icp_lib.load_matrix(datasets.path(mname))
    p = icp_lib.load_matrix(datasets.path(pname))
    with icp_lib.Context(0) as c:
        c.set_model(m)
        c.set_scene(p)
        res, errs = c.run(iters)
        final = c.get_scene()
    assert res.iterations == out["iterations"]
    np.testing.assert_allclose(errs, out["err"], rtol=1e-9)
    np.testing.assert_allclose(final.sum(axis=0), out["final_sum"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(final[0], out["final_head"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(final[-1], out["final_tail"], rtol=0, atol=1e-9)


def test_comm_info(icp_lib):
    """icp_get_comm_info: what bench.py's per_rank records for every rank of a multi-GPU line."""
    with icp_lib.Context(0) as c:
        info = c.comm_info()
        assert info["comm_count"] is None and info["comm_rank"] == 0
        bus = info["pci_bus_id"]
        assert len(bus) >= 7 and ":" in bus  # e.g. 0000:05:00.0
    with icp_lib.Context(0, icp_lib.NN_CERTIFIED, rank=0, world_size=1, rccl_id=icp_lib.rccl_unique_id()) as c:
        info = c.comm_info()
        assert info["comm_count"] == 1 and info["comm_rank"] == 0 and info["pci_bus_id"] == bus


def test_closest_matrix_mapped_buffer_limit(icp_lib):
    """Queries up to the mapped buffer's size take the one-launch LDS search of a small model
    (closest_lds: 6.5 doubles per query); 65,536 queries against cow need more than the buffer
    holds and must take the staged path -- both bitwise equal to the cascade."""
    m = icp_lib.load_matrix(datasets.path("cow_ref"))
    rng = np.random.default_rng(9)
    lo, hi = m.min(axis=0), m.max(axis=0)
    for n in (60000, 60494, 60495, 65536):
        p = rng.uniform(lo, hi, size=(n, 3))
        with icp_lib.Context(0) as c:
            c.set_model(m)
            y, idx = c.closest_matrix(p)
        with icp_lib.Context(0) as c:
            c.set_nn_variant(icp_lib.VARIANT_VALU)  # an explicit variant: the cascade
            c.set_model(m)
            y2, idx2 = c.closest_matrix(p)
        assert np.array_equal(idx, idx2), n
        assert np.array_equal(y, y2), n
        assert np.array_equal(y, m[idx]), n
