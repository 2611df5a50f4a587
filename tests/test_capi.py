"""CPU-side checks of the product C-ABI (libicp_hip.so): it loads without a GPU, exports
every function include/icp_capi.h declares, and its host-only pieces (Horn solve, quirk,
sharding, synthetic generator, CSV I/O) match the oracle.  No device compute here."""
import os
import re

import numpy as np
import pytest

import datasets

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RNG = np.random.default_rng(7)


def declared_functions():
    src = open(os.path.join(ROOT, "include", "icp_capi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(icp_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol(icp_lib):
    names = declared_functions()
    assert len(names) >= 25
    L = icp_lib.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(icp_lib.EXPORTED) == names


def test_no_device_fails_loudly(icp_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(icp_lib.ICPError) as ei:
        icp_lib.Context()
    assert ei.value.code == icp_lib.ICP_E_NO_DEVICE


def test_strerror_messages_match_reference(icp_lib):
    assert icp_lib.strerror(icp_lib.ICP_E_SIZE_MISMATCH) == \
        "Point sets need to have the same number of points."  # cpu.cc:45
    assert icp_lib.strerror(icp_lib.ICP_E_TOO_FEW_POINTS) == "Need at least 4 point pairs"


def test_horn_solve_matches_oracle(icp_lib, oracle):
    for trial in range(30):
        n = 50
        p = RNG.normal(size=(n, 3))
        ang = RNG.uniform(-np.pi, np.pi)
        ax = RNG.normal(size=3); ax /= np.linalg.norm(ax)
        K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        R = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
        y = 1.3 * p @ R.T + RNG.normal(size=3) + RNG.normal(scale=0.05, size=(n, 3))
        al = oracle.find_alignment(p, y)
        s, Rh, t = icp_lib.horn_solve(al.S, al.mu_p, al.mu_y, al.d_caps, al.sp)
        np.testing.assert_allclose(Rh, np.array(al.R).reshape(3, 3), atol=1e-12)
        assert s == al.s  # same formula, same rounding
        np.testing.assert_allclose(t, np.array(al.t), atol=1e-12)


def test_max_element_index_is_the_reference_quirk(icp_lib, oracle):
    for _ in range(200):
        ev = RNG.normal(size=4)
        assert icp_lib.max_element_index(ev) == oracle.max_element_index(ev)


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (7, 2), (2903, 2), (1 << 20, 8), (1 << 23, 8), (10, 16)])
def test_shard_range_partitions(icp_lib, n, world):
    nxt = 0
    counts = []
    for r in range(world):
        b, c = icp_lib.shard_range(n, r, world)
        assert b == nxt
        nxt = b + c
        counts.append(c)
    assert nxt == n and max(counts) - min(counts) <= 1


def test_synthetic_pair(icp_lib):
    m, p = icp_lib.synthetic_pair(4096, seed=42)
    m2, p2 = icp_lib.synthetic_pair(4096, seed=42)
    np.testing.assert_array_equal(m, m2)
    assert np.all(np.abs(m) <= 1.0)
    np.testing.assert_array_equal(m.astype(np.float32).astype(np.float64), m)  # fp32-representable
    np.testing.assert_array_equal(p.astype(np.float32).astype(np.float64), p)
    # scene = R m + t (5 deg about (1,2,3)), same point order
    ax = np.array([1.0, 2.0, 3.0]) / np.sqrt(14.0)
    th = np.deg2rad(5.0)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    np.testing.assert_allclose(p, m @ R.T + [0.05, -0.03, 0.02], atol=1e-7)


@pytest.mark.parametrize("name", datasets.NAMES)
def test_load_matrix_bitwise_equals_oracle(icp_lib, oracle, name):
    a = icp_lib.load_matrix(datasets.path(name))
    b = oracle.load_matrix(datasets.path(name))
    assert a.shape == b.shape
    np.testing.assert_array_equal(a, b)


def test_load_matrix_edge_cases(icp_lib, oracle, tmp_path):
    f = tmp_path / "c.txt"
    f.write_text("Points_0,Points_1,Points_2\n1.5,2,3\n-4e-3,5,6,7\n\n8,9\n +1e2, -2,0x10\n")
    np.testing.assert_array_equal(icp_lib.load_matrix(str(f)), oracle.load_matrix(str(f)))
    with pytest.raises(icp_lib.ICPError):
        icp_lib.load_matrix(str(tmp_path / "missing.txt"))


def test_write_matrix_byte_identical(icp_lib, oracle, tmp_path):
    x = np.concatenate([RNG.normal(size=(100, 3)) * 10.0 ** RNG.integers(-8, 8, size=(100, 1)),
                        [[0.0, -0.0, 1e300]]])
    a, b = tmp_path / "a.txt", tmp_path / "b.txt"
    icp_lib.write_matrix(str(a), x)
    oracle.lib().oracle_write_matrix(str(b).encode(), oracle._dp(np.ascontiguousarray(x)), x.shape[0])
    assert a.read_bytes() == b.read_bytes()
    assert a.read_text().splitlines()[0] == "Points_0,Points_1,Points_2"
