"""The fast f16 split (icp_mfma16.h split_f16: fp32 round-to-odd, then f16 round-to-nearest)
equals the direct correctly rounded (_Float16) conversions bit for bit on the GPU.

Every f16 operand of the filters (query and model images, bundle and group bounds) goes
through split_f16, and the certificates' error budgets assume correctly rounded halves; the
faster form must therefore give the same bits.  tools/split_probe.hip converts 2^26 doubles
(wide-range values, values within 2^-50 ulp of an f16 rounding tie, scaled-coordinate-like
values, random finite bit patterns) both ways on the device and counts mismatches.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "split_probe.hip")
BIN = os.path.join(ROOT, "tools", "split_probe")


@pytest.mark.gpu
def test_fast_split_equals_direct_conversion():
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < os.path.getmtime(SRC):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-ffp-contract=off",
                        "-fno-honor-nans", "-mno-amdgpu-ieee", "-o", BIN, SRC], check=True, capture_output=True)
    out = subprocess.run([BIN], check=True, capture_output=True, text=True, timeout=120).stdout
    m = re.search(r"SPLIT n=(\d+) bad=(\d+)", out)
    assert m, out
    assert int(m.group(1)) == 1 << 26
    assert int(m.group(2)) == 0
