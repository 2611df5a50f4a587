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


def _fuzz_token(rng):
    """A number spelled one of the ways a CSV row may carry it (decimal, exponent, long
    mantissa, hex, inf/nan, padding, signs) or junk."""
    v = rng.normal() * 10.0 ** rng.integers(-30, 30)
    k = rng.integers(0, 16)
    if k < 6:
        return f"{v:.{rng.integers(1, 18)}g}"
    if k == 6:
        return repr(v)
    if k == 7:
        return f"{v:.{rng.integers(0, 25)}f}"
    if k == 8:
        return float(v).hex()
    if k == 9:
        return str(rng.choice(["inf", "-inf", "nan", "Infinity", "-0", "0", "-0.0", "1e400", "-1e-400",
                               "4.9e-324", "2.2250738585072014e-308", "9007199254740993", "1e22", "1e23"]))
    if k == 10:
        return " " * int(rng.integers(1, 3)) + f"{v:.6g}"
    if k == 11:
        return "+" + f"{abs(v):.8g}"
    if k == 12:
        return str(rng.integers(-10**6, 10**6)) + "." + "0" * int(rng.integers(0, 30)) + str(rng.integers(0, 10**6))
    if k == 13:
        return f"{v:.5e}".replace("e", "E")
    if k == 14:
        return str(rng.choice(["", "-", ".", "1e", "1e+", "abc", "0x", "00x1", ".5", "-.5", "5.", "1.5e+0x"]))
    return "0" * int(rng.integers(1, 5)) + f"{abs(v):.7g}"


def test_load_matrix_fuzz_bitwise_equals_sscanf(icp_lib, oracle, tmp_path):
    # the oracle parses with sscanf("%lf,%lf,%lf") (load.cc:27); the product's parser takes an
    # exact fast path for plain decimals and strtod for the rest: bit-identical either way
    rng = np.random.default_rng(5)
    rows = []
    for _ in range(4000):
        toks = [_fuzz_token(rng) for _ in range(int(rng.integers(0, 5)))]
        sep = str(rng.choice([",", ",", ",", ", ", ";"]))
        rows.append(sep.join(toks) + str(rng.choice(["", "", "\r"])))
    f = tmp_path / "fuzz.txt"
    f.write_bytes(("Points_0,Points_1,Points_2\n" + "\n".join(rows) + "\n").encode())
    a, b = icp_lib.load_matrix(str(f)), oracle.load_matrix(str(f))
    assert a.shape == b.shape
    np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))


def test_load_matrix_multithreaded_large(icp_lib, oracle, tmp_path):
    # > 1 MiB per thread: the chunked parallel path, rows split across chunk boundaries
    x = RNG.normal(size=(300000, 3)) * 10.0 ** RNG.integers(-5, 5, size=(300000, 1))
    f = tmp_path / "big.txt"
    with open(f, "w") as fh:
        fh.write("Points_0,Points_1,Points_2\n")
        fh.writelines(f"{a:.17g},{b:.9g},{c!r}\n" for a, b, c in x)
    a, b = icp_lib.load_matrix(str(f)), oracle.load_matrix(str(f))
    assert a.shape == (300000, 3)
    np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))
    out1, out2 = tmp_path / "o1.txt", tmp_path / "o2.txt"
    icp_lib.write_matrix(str(out1), a)
    oracle.lib().oracle_write_matrix(str(out2).encode(), oracle._dp(np.ascontiguousarray(a)), a.shape[0])
    assert out1.read_bytes() == out2.read_bytes()


def test_write_matrix_byte_identical(icp_lib, oracle, tmp_path):
    x = np.concatenate([RNG.normal(size=(100, 3)) * 10.0 ** RNG.integers(-8, 8, size=(100, 1)),
                        [[0.0, -0.0, 1e300]]])
    a, b = tmp_path / "a.txt", tmp_path / "b.txt"
    icp_lib.write_matrix(str(a), x)
    oracle.lib().oracle_write_matrix(str(b).encode(), oracle._dp(np.ascontiguousarray(x)), x.shape[0])
    assert a.read_bytes() == b.read_bytes()
    assert a.read_text().splitlines()[0] == "Points_0,Points_1,Points_2"


def _rot(ax, ang):
    ax = np.asarray(ax, float) / np.linalg.norm(ax)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


@pytest.mark.parametrize("case", ["scaled_small", "scaled_large", "half_turn", "identity", "planar",
                                  "cube_corners", "line", "two_points_dup", "noise_only"])
def test_horn_solve_edge_cases(icp_lib, oracle, case):
    """The Horn step's eigen-solver (characteristic-polynomial path, Jacobi fallback for a
    near-multiple largest eigenvalue) against the oracle's Jacobi: the same rotation where it
    is unique, and the same residual where it is not (a line's spin is undetermined)."""
    rng = np.random.default_rng(hash(case) % 2**32)
    n = 40
    p = rng.normal(size=(n, 3))
    R0 = _rot(rng.normal(size=3), 0.7)
    if case == "scaled_small":
        p *= 1e-5
    elif case == "scaled_large":
        p = p * 1e5 + 3e6
    elif case == "half_turn":
        R0 = _rot([0.3, -0.5, 0.8], np.pi)
    elif case == "identity":
        R0 = np.eye(3)
    elif case == "planar":
        p[:, 2] = 0.0
        R0 = _rot([0, 0, 1], 0.4)
    elif case == "cube_corners":
        p = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], float)
    elif case == "line":
        p = np.outer(np.linspace(-1, 1, n), [1.0, 2.0, -0.5])
    elif case == "two_points_dup":
        p = np.array([[1.0, 0, 0], [1.0, 0, 0], [-1.0, 0, 0], [-1.0, 0, 0], [0, 1.0, 0]])
    y = p @ R0.T + np.array([0.1, -0.2, 0.3])
    if case == "noise_only":
        y = rng.normal(size=(n, 3))
    al = oracle.find_alignment(p, y)
    s, Rh, t = icp_lib.horn_solve(al.S, al.mu_p, al.mu_y, al.d_caps, al.sp)
    Rh = np.asarray(Rh).reshape(3, 3)
    np.testing.assert_allclose(Rh @ Rh.T, np.eye(3), atol=1e-12)
    assert abs(np.linalg.det(Rh) - 1.0) < 1e-12
    def resid(R_, s_, t_):
        return float(((y - (s_ * p @ np.asarray(R_).reshape(3, 3).T + np.asarray(t_))) ** 2).sum())
    r_ours, r_ref = resid(Rh, s, t), resid(al.R, al.s, al.t)
    scale = float((y ** 2).sum()) + 1.0
    assert abs(r_ours - r_ref) <= 1e-9 * scale, (r_ours, r_ref)
    if case not in ("line", "two_points_dup", "noise_only"):
        np.testing.assert_allclose(Rh, np.array(al.R).reshape(3, 3), atol=1e-9)
