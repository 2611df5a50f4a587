"""bench.py's multi-GPU evidence (CPU only): every rank's per_rank entry carries its RCCL
communicator's size and rank and its device's PCI bus id (icp_get_comm_info), and rank 0
refuses to report an RCCL line whose ranks are not N distinct GPUs of one N-rank communicator."""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def rec(rank, count, crank, bus):
    return bench.rank_record(rank, {"comm_count": count, "comm_rank": crank, "pci_bus_id": bus}, 3.5, 0.02,
                             131072, 30)


def buses(n):
    return [f"0000:{0x05 + 0x10 * k:02x}:00.0" for k in range(n)]


def test_rccl_eight_distinct_gpus_pass():
    pr = [rec(r, 8, r, b) for r, b in enumerate(buses(8))]
    assert bench.check_devices(pr, 8, rccl=True) is None
    assert set(pr[0]) >= {"rank", "filter_ms", "allreduce_ms_per_iter", "comm_count", "comm_rank", "pci_bus_id"}


@pytest.mark.parametrize("case", ["dup_bus", "wrong_count", "no_comm", "wrong_rank", "missing_rank"])
def test_rccl_bad_lines_fail(case):
    b = buses(4)
    pr = [rec(r, 4, r, b[r]) for r in range(4)]
    if case == "dup_bus":
        pr[3]["pci_bus_id"] = b[0]
    elif case == "wrong_count":
        pr[1]["comm_count"] = 2
    elif case == "no_comm":
        pr[2]["comm_count"] = None
    elif case == "wrong_rank":
        pr[2]["comm_rank"] = 1
    else:
        pr = pr[:3]
    assert bench.check_devices(pr, 4, rccl=True) is not None


def test_host_reduce_rehearsal_allows_one_gpu():
    """The gloo rehearsal (ICP_BENCH_HOST_REDUCE=1) runs several ranks on one GPU without RCCL:
    comm_count is null and the bus ids repeat, which is what it is."""
    pr = [rec(r, None, r, "0000:05:00.0") for r in range(2)]
    assert bench.check_devices(pr, 2, rccl=False) is None


def test_committed_rehearsal_lines_carry_device_fields():
    """The committed N>1 rehearsal lines (profiles/*dist*rehearsal*.log) of this round's bench
    carry the per-rank device fields, parse, and pass the device check they ran under."""
    logs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r03*dist*rehearsal*.log")))
    assert logs, "no round-3 rehearsal log committed under profiles/"
    for path in logs:
        line = [ln for ln in open(path) if ln.startswith("{") and '"metric"' in ln][-1]
        out = json.loads(line)
        world = out["n_gpus"]
        pr = out["per_rank"]
        assert len(pr) == world > 1
        for r in pr:
            assert {"comm_count", "comm_rank", "pci_bus_id", "filter_ms", "allreduce_ms_per_iter"} <= set(r)
        host = "gloo host all-reduce" in out["config"]["parallelism"]
        if host:
            assert all(r["comm_count"] is None for r in pr)
        assert bench.check_devices(pr, world, rccl=not host) is None
        assert "device_error" not in out
