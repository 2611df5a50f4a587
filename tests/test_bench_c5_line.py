"""The C5 bench line describes itself (CPU only).

bench.py at --points 8388608 labels its metric and workload C5 and, for rank 0's shard of the
8-way run, takes the dominant kernel's HBM bytes per launch from the committed C5-shard capture
(profiles/<tag>_c5shard_pmc_traffic.json, tools/gpu_round.sh c5pmc).  The newest committed C5
line (the 8-rank flow rehearsed on one GPU, tools/gpu_round.sh c5dist8) must carry the label, the
traffic and every rank's filter and tail times.
"""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c5_lines():
    out = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "**", "*.log"), recursive=True):
        try:
            lines = open(path).read().splitlines()
        except (OSError, UnicodeDecodeError):
            continue
        for line in lines:
            if line.startswith("{") and '"n_model": 8388608' in line:
                out.append((os.path.getmtime(path), path, json.loads(line)))
    return sorted(out, key=lambda t: t[1])


def test_c5_line_is_labelled_and_carries_traffic():
    lines = [x for x in _c5_lines() if "traffic_source" in json.dumps(x[2]) and x[2].get("n_gpus") == 8]
    lines = [x for x in lines if (x[2]["roofline"].get("traffic_source") or "").endswith("_c5shard_pmc_traffic.json")]
    if not lines:
        pytest.skip("no committed 8-rank C5 line with the C5-shard traffic yet")
    _, path, d = lines[-1]
    assert "C5" in d["metric"] and "8388608" in d["metric"], path
    assert d["config"]["workload"].startswith("C5"), path
    r = d["roofline"]
    assert r["traffic"] and r["traffic"] > 0
    src = json.load(open(os.path.join(ROOT, r["traffic_source"])))
    key = r["kernel"].split(" ")[0]
    assert src["kernels"][key]["traffic_bytes_per_launch"] == r["traffic"]
    ranks = d["per_rank"]
    assert sorted(x["rank"] for x in ranks) == list(range(8))
    for x in ranks:
        assert x["filter_ms"] > 0 and x["tail_ms"] is not None and x["n_scene_local"] == 8388608 // 8


def test_bench_traffic_lookup_keeps_workloads_apart():
    """pmc_traffic(kernel) reads only this bench's C4 captures (<tag>_pmc_traffic.json), never a
    configuration's (<tag>_<cfg>_pmc_traffic.json), and pmc_traffic(kernel, cfg) only that cfg's."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import importlib
    bench = importlib.import_module("bench")
    for cfg in ("", "c3", "grid", "c5shard"):
        for kernel in ("nn_grid_seeded_kernel", "icp_persistent_mid_kernel", "transform_err_kernel"):
            b, src = bench.pmc_traffic(kernel, cfg)
            if src is None:
                continue
            name = os.path.basename(src)
            if cfg:
                assert name.endswith(f"_{cfg}_pmc_traffic.json")
            else:
                assert name.count("_") == 2
