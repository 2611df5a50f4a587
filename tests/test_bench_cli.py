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
