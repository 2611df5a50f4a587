"""Bundled point-cloud fixtures (the reference's data_students/*.txt, gzip'ed byte-exact).

The reference ships these CSV clouds as its only data (data_students/README.md:9-21); the
GPU box has no /root/reference, so they travel as tests/golden/data/*.txt.gz and are
decompressed on first use into a per-user cache directory.
"""
from __future__ import annotations

import gzip
import os
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "data")
NAMES = ["cow_ref", "cow_tr1", "cow_tr2", "horse_ref", "horse_tr1", "horse_tr2", "bun000", "bun045"]

_CACHE = os.path.join(tempfile.gettempdir(), f"icp_amd_data_{os.getuid()}")


def path(name: str) -> str:
    """Filesystem path of the decompressed `<name>.txt`."""
    os.makedirs(_CACHE, exist_ok=True)
    out = os.path.join(_CACHE, name + ".txt")
    if not os.path.exists(out):
        tmp = out + f".{os.getpid()}.tmp"
        with gzip.open(os.path.join(DATA, name + ".txt.gz"), "rb") as f, open(tmp, "wb") as g:
            g.write(f.read())
        os.replace(tmp, out)
    return out
