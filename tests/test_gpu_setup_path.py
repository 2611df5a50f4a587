"""The registration's setup path (icp_engine.hip: scene_from_aos, set_model_staged; icp_order.hip:
launch_slot_order_aos; icp_grid.hip: grid_rep_kernel, nn_grid_cell_seed_kernel).

The reference's registration is the GPU::ICP constructor (src/GPU/gpu.hh:44-56: the clouds'
copies) and then find_corresponding_opti (src/GPU/gpu.cc:52-83) from an unseeded first search.
Here a scene of the slot-order size is sorted and gathered straight from its AoS array at
icp_set_scene, and the run's first search takes the seeded grid pass from cell seeds.  Neither
may change a result: the same slot order (stable sort of the same keys from file order), and the
exact first minimum over a complete box whatever the seed.  Cases:

  * icp_set_scene (host array) and icp_set_scene_device (a device tensor): bit for bit;
  * the scene set before the model and after it: bit for bit (a slot-ordered scene goes back to
    file order when the model changes, and the run sorts it by the new model's box);
  * the cell-seeded first search against the ring search (ICP_CELL_SEED=0, a subprocess: the
    switch is read once), on the AUTO and GRID variants: the same trajectory bit for bit, and the
    first search's indices against the oracle's brute force -- including a scene displaced by a
    model extent, whose queries sit in border cells, many of them empty (stand-in seeds).
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch  # (before the first HIP call of the session: torch then sees the device)

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def trajectory(ctx, iters=8):
    ctx.set_index_digest(iters)
    res, errs = ctx.run(iters, -1.0)
    return dict(errs=errs, dig=ctx.index_digest(iters), scene=ctx.get_scene(), s=res.s,
                R=np.array(res.R[:]), t=np.array(res.t[:]))


def assert_same(a, b):
    for k in ("errs", "dig", "scene", "R", "t"):
        assert np.array_equal(a[k], b[k]), k
    assert a["s"] == b["s"]


def test_scene_device_matches_host_upload(amd):
    n = 1 << 16
    m, p = amd.synthetic_pair(n, seed=21)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        a = trajectory(ctx)
    dm = torch.from_numpy(m).to("cuda:0")
    dp = torch.from_numpy(p).to("cuda:0")
    torch.cuda.synchronize()
    with amd.Context(0) as ctx:
        ctx.set_model_device(dm.data_ptr(), n)
        ctx.set_scene_device(dp.data_ptr(), n)
        b = trajectory(ctx)
    assert_same(a, b)


@pytest.mark.parametrize("form", ["any_stream", "producer_stream"])
def test_device_arrays_written_on_another_stream(amd, form):
    """The device-array setters read the caller's array after the work that writes it, with no
    manual synchronisation: the clouds are zeros until a copy queued on a side stream
    behind a ~10 ms spin fills them.  icp_set_*_device orders after every stream (device
    synchronisation); icp_set_*_device_stream after the given producer stream."""
    n = 1 << 16
    m, p = amd.synthetic_pair(n, seed=21)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        a = trajectory(ctx)
    dm = torch.zeros((n, 3), dtype=torch.float64, device="cuda:0")
    dp = torch.zeros((n, 3), dtype=torch.float64, device="cuda:0")
    hm = torch.from_numpy(m).pin_memory()
    hp = torch.from_numpy(p).pin_memory()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(20_000_000)  # (cycles: the copies land well after the calls are made)
        dm.copy_(hm, non_blocking=True)
        dp.copy_(hp, non_blocking=True)
    with amd.Context(0) as ctx:
        if form == "any_stream":
            ctx.set_model_device(dm.data_ptr(), n)
            ctx.set_scene_device(dp.data_ptr(), n)
        else:
            ctx.set_model_device(dm.data_ptr(), n, stream=side.cuda_stream)
            ctx.set_scene_device(dp.data_ptr(), n, stream=side.cuda_stream)
        b = trajectory(ctx)
    assert_same(a, b)


def test_scene_stream_setter_is_stream_ordered(amd):
    """icp_set_scene_device_stream returns before the producer's copy has landed (no host wait: the
    context's stream waits for the producer's event) and the run still reads the copied scene."""
    n = 1 << 16
    m, p = amd.synthetic_pair(n, seed=21)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        a = trajectory(ctx)
    dm = torch.from_numpy(m).to("cuda:0")
    dp = torch.zeros((n, 3), dtype=torch.float64, device="cuda:0")
    hp = torch.from_numpy(p).pin_memory()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with amd.Context(0) as ctx:
        ctx.set_model_device(dm.data_ptr(), n, stream=side.cuda_stream)
        done = torch.cuda.Event()
        with torch.cuda.stream(side):
            torch.cuda._sleep(400_000_000)  # (cycles: ~0.2 s)
            dp.copy_(hp, non_blocking=True)
            done.record(side)
        ctx.set_scene_device(dp.data_ptr(), n, stream=side.cuda_stream)
        assert not done.query()  # the setter did not wait for the producer
        b = trajectory(ctx)
    assert_same(a, b)


def test_scene_before_model_matches_after(amd):
    n = 1 << 16
    m0, _ = amd.synthetic_pair(n, seed=3)
    m, p = amd.synthetic_pair(n, seed=4, angle_deg=7.0)
    with amd.Context(0) as ctx:  # the scene sorted by the first model's box, then a new model
        ctx.set_model(0.5 * m0 + 0.25)
        ctx.set_scene(p)
        ctx.set_model(m)
        a = trajectory(ctx)
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        b = trajectory(ctx)
    assert_same(a, b)


CELL_SEED_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import icp_amd
out = {}
n = 1 << 16
rng = np.random.default_rng(17)
m = rng.uniform(-1, 1, size=(n, 3))
cases = {"near": icp_amd.synthetic_pair(n, seed=8)[1], "far": m @ np.diag([1.0, -1.0, 1.0]) + [1.9, 0.4, -0.2]}
for name, p in cases.items():
    for variant in (icp_amd.VARIANT_AUTO, icp_amd.VARIANT_GRID):
        with icp_amd.Context(0) as ctx:
            ctx.set_nn_variant(variant)
            ctx.set_model(m)
            ctx.set_scene(p)
            ctx.run(1, -1.0)
            key = f"{name}_{variant}"
            out[key + "_idx1"] = ctx.get_indices()
            ctx.set_index_digest(6)
            _, errs = ctx.run(6, -1.0)
            out[key + "_errs"] = errs
            out[key + "_dig"] = ctx.index_digest(6)
            out[key + "_scene"] = ctx.get_scene()
np.savez(sys.argv[2], **out)
print("cell seed ok")
"""


def run_cell_seed(tmp_path, flag):
    out = str(tmp_path / f"cell_seed_{flag}.npz")
    env = dict(os.environ, ICP_CELL_SEED=flag)
    r = subprocess.run([sys.executable, "-c", CELL_SEED_SCRIPT, os.path.join(ROOT, "iterative-closest-point_amd"), out],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "cell seed ok" in r.stdout, r.stdout + r.stderr
    return dict(np.load(out))


def test_cell_seeded_first_search_matches_ring_search(amd, oracle, tmp_path):
    cell = run_cell_seed(tmp_path, "1")
    ring = run_cell_seed(tmp_path, "0")
    assert cell.keys() == ring.keys()
    for k in cell:
        assert np.array_equal(cell[k], ring[k]), k
    # the first search (from the scene as given) against the brute force
    n = 1 << 16
    rng = np.random.default_rng(17)
    m = rng.uniform(-1, 1, size=(n, 3))
    p_near = amd.synthetic_pair(n, seed=8)[1]
    p_far = m @ np.diag([1.0, -1.0, 1.0]) + [1.9, 0.4, -0.2]
    sel = np.sort(np.random.default_rng(5).choice(n, 512, replace=False))
    for name, p in (("near", p_near), ("far", p_far)):
        _, ref = oracle.closest_blocked(p[sel], m)
        for variant in (amd.VARIANT_AUTO, amd.VARIANT_GRID):
            assert np.array_equal(cell[f"{name}_{variant}_idx1"][sel], ref), (name, variant)
