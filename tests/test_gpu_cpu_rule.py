"""The reference CPU path's NN rule on the GPU engine (ICP_NN_RULE_CPU_SQRT, the `icp` binary).

src/cpu.cc:17-22 takes the first minimum of sqrt((pow(dx,2) + pow(dy,2)) + pow(dz,2)) with
libm's pow; the GPU path (compute.cu:112-117) the first minimum of the squared distance.  They
differ only at near ties: on bunny (bun000 / bun045) at queries 8277, 15594 and 20678 of the
first search.  The engine finds each query's near-tie window on the device and evaluates the
reference's CPU arithmetic with libm on the host for exactly those candidates.  Checked against
the oracle built with real libm pow calls (oracle/Makefile: -fno-builtin-pow):
  * bunny's first search, all 40,097 queries: bit-exact (tests/golden/bun045_cpu_rule_idx0.npz);
  * bunny, the 50 ICP iterations of BASELINE config C2 (allow_unequal): err rtol 1e-9, s/R/t
    atol 1e-9 (tests/golden/cpu_rule.json, made by tests/golden/make_cpu_rule.py) -- under the
    squared rule the same run agrees only to ~1e-3;
  * cow (no near ties): the two rules give bit-identical runs;
  * a lattice model with half-integer queries (exact ties everywhere): bit-exact vs the oracle.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(ROOT, "iterative-closest-point_amd", "build")
FX = json.load(open(os.path.join(HERE, "golden", "cpu_rule.json")))
TIES = [8277, 15594, 20678]


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


@pytest.fixture(scope="module")
def bunny(amd):
    return amd.load_matrix(datasets.path("bun000")), amd.load_matrix(datasets.path("bun045"))


def test_bunny_first_search_bit_exact(amd, bunny):
    m, p = bunny
    want = np.load(os.path.join(HERE, "golden", "bun045_cpu_rule_idx0.npz"))["idx0"]
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        _, sq = ctx.closest_matrix(p)
        ctx.set_nn_rule(amd.RULE_CPU_SQRT)
        ctx.reset_stats()
        y, cpu = ctx.closest_matrix(p)
        st = ctx.stats()
    np.testing.assert_array_equal(cpu, want)
    assert np.nonzero(cpu != sq)[0].tolist() == TIES
    assert st["cpu_rule_changed"] == len(TIES) and st["cpu_rule_ties"] >= len(TIES)
    np.testing.assert_array_equal(y, m[cpu])


@pytest.mark.parametrize("variant_name", ["VARIANT_AUTO", "VARIANT_GRID", "VARIANT_VALU"])
def test_bunny_icp_run_matches_cpu_rule_oracle(amd, bunny, variant_name):
    m, p = bunny
    g = FX["bunny"]
    with amd.Context(0) as ctx:
        ctx.set_nn_variant(getattr(amd, variant_name))
        ctx.set_nn_rule(amd.RULE_CPU_SQRT)
        ctx.set_allow_unequal(True)
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(g["max_iter"], g["threshold"])
        fin = ctx.get_scene()
    assert res.iterations == g["iterations"]
    np.testing.assert_allclose(errs, g["err"], rtol=1e-9)
    np.testing.assert_allclose(res.s, g["s"][-1], rtol=0, atol=1e-9)
    np.testing.assert_allclose(np.array(res.R).reshape(3, 3), np.array(g["R"][-1]), rtol=0, atol=1e-9)
    np.testing.assert_allclose(res.t, g["t"][-1], rtol=0, atol=1e-9)
    np.testing.assert_allclose(fin.sum(axis=0), g["final_sum"], rtol=1e-9)
    np.testing.assert_allclose(fin[:4], g["final_head"], rtol=0, atol=1e-9)


def test_cow_rules_agree_bitwise(amd):
    m = amd.load_matrix(datasets.path("cow_ref"))
    p = amd.load_matrix(datasets.path("cow_tr1"))
    out = {}
    for rule in (amd.RULE_SQUARED, amd.RULE_CPU_SQRT):
        with amd.Context(0) as ctx:
            ctx.set_nn_rule(rule)
            ctx.set_model(m)
            ctx.set_scene(p)
            res, errs = ctx.run(20)
            out[rule] = (res.iterations, errs, ctx.get_scene())
    assert out[0][0] == out[1][0] == FX["cow_tr1"]["iterations"]
    np.testing.assert_array_equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][2], out[1][2])
    np.testing.assert_allclose(out[1][1], FX["cow_tr1"]["err"], rtol=1e-9)


def test_lattice_ties_bit_exact(amd, oracle):
    rng = np.random.default_rng(11)
    g = np.arange(-6, 7, dtype=float) * 0.1  # 0.1 is inexact: ties up to rounding everywhere
    m = np.stack(np.meshgrid(g, g, g[:6], indexing="ij"), axis=-1).reshape(-1, 3)
    m = m[rng.permutation(m.shape[0])]
    q = m[rng.integers(0, m.shape[0], 600)] + 0.05
    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_nn_rule(amd.RULE_CPU_SQRT)
        _, got = ctx.closest_matrix(q)
    _, want = oracle.closest(q, m, oracle.NN_CPU_SQRT)
    np.testing.assert_array_equal(got, want)


def test_icp_cli_keeps_the_cpu_rule(tmp_path):
    """`icp` (src/main.cc) runs the CPU rule, `icp-gpu` the squared one: on bunny their
    [ICP] lines differ, and `icp`'s follow the CPU-rule oracle."""
    ref, scene = datasets.path("bun000"), datasets.path("bun045")
    g = FX["bunny"]
    lines = {}
    for exe in ("icp", "icp-gpu"):
        r = subprocess.run([os.path.join(BUILD, exe), ref, scene, str(g["max_iter"]), "--allow-unequal",
                            "--threshold", "-1"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines[exe] = [l for l in r.stderr.splitlines() if l.startswith("[ICP]")]
    want = [f"[ICP] iteration number {i} | error value = {e:g}" for i, e in enumerate(g["err"])]
    assert lines["icp"] == want
    assert lines["icp-gpu"] != want
