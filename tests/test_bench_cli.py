"""bench.py's command line under the driver's launcher (CPU only: argument parsing, no engine).

The multi-GPU runs go through `python -m torch.distributed.run ... bench.py --gpus N ...`; that
launcher's own parser must hand every bench option to bench.py (a bare `--n` was taken as an
ambiguous prefix of --nnodes / --nproc-per-node and the launch stopped).
"""
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
BENCH_FLAGS = ["--gpus", "8", "--steps", "30", "--warmup", "2", "--points", "8388608", "--no-cow", "--no-cases",
               "--no-cpu-baseline", "--variant", "auto", "--nn", "certified"]


def test_torchrun_passes_every_bench_flag_through():
    from torch.distributed.run import get_args_parser
    args = get_args_parser().parse_args(["--nnodes=1", "--nproc-per-node", "8", "--master-addr", "127.0.0.1",
                                         "--master-port", "29500", "bench.py"] + BENCH_FLAGS)
    assert args.training_script == "bench.py"
    assert args.training_script_args == BENCH_FLAGS


def test_bench_help_lists_points_and_keeps_n_alias():
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--help"], capture_output=True, text=True,
                         timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    assert re.search(r"--points N, --n N", out.stdout), out.stdout


@pytest.mark.parametrize("doc", ["README.md", "DESIGN.md"])
def test_documented_torchrun_commands_parse(doc):
    """Every `bench.py` line of a documented torchrun command passes the launcher's parser."""
    from torch.distributed.run import get_args_parser
    text = (ROOT / doc).read_text()
    cmds = re.findall(r"torch\.distributed\.run ([^\n]*\\\n[^\n]*|[^\n]*)", text)
    checked = 0
    for c in cmds:
        argv = c.replace("\\\n", " ").split("#")[0].split()
        if "bench.py" not in argv:
            continue
        argv = [a for a in argv if "$" not in a]
        args = get_args_parser().parse_args(argv)
        assert args.training_script == "bench.py"
        checked += 1
    assert checked > 0


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_dtype_describes_what_ran():
    """The line's dtype is composed from one registration's counters (icp_stats), not fixed text:
    a C4 registration that ran only grid searches names the grid kernel and its certified share and
    no bundle filter; one whose early searches took the bundle cascade names both."""
    bench = _bench_module()
    grid_only = {"run_grid_searches": 30, "run_bundle_searches": 0, "run_certified": 750, "run_walked": 250}
    d = bench.path_description(grid_only)
    assert "30 exact fp64 grid searches" in d and bench.grid_kernel() in d and "75%" in d
    assert "bundle" not in d
    mixed = {"run_grid_searches": 27, "run_bundle_searches": 3, "run_certified": 0, "run_walked": 0}
    d = bench.path_description(mixed)
    assert "27 exact fp64 grid searches" in d and "3 searches through the f16" in d


def test_committed_bench_line_dtype_matches_its_counters():
    """The round-6 GPU bench lines (profiles/r06*/*bench*.log) carry step_paths, and the last one's
    dtype is the description of exactly those counters."""
    import json
    logs = sorted(ROOT.glob("profiles/r06*/*bench*.log"))
    lines = [json.loads(x) for f in logs for x in f.read_text().splitlines() if x.startswith("{")]
    lines = [x for x in lines if "step_paths" in x]
    if not lines:
        pytest.skip("no round-6 bench line with step_paths committed yet")
    bench = _bench_module()
    last = lines[-1]
    sp = {k: last["step_paths"][k] for k in ("run_grid_searches", "run_bundle_searches", "run_certified",
                                             "run_walked")}
    assert last["dtype"] == "f64 (" + bench.path_description(sp) + ")"
