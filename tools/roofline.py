#!/usr/bin/env python3
"""Recompute every roofline figure bench.py reports from the committed profiles.

    python tools/roofline.py [--tag r02a] [--n 1048576] [--world 1]

Inputs (both written by tools/gpu_round.sh on the GPU box, then copied into profiles/):
  profiles/<tag>_bench_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `bench.py --no-cases`
  profiles/<tag>_pmc_traffic.json         tools/pmc_summary.py over separate FETCH_SIZE / WRITE_SIZE
                                          passes of the same command (FETCH_SIZE doubled, gfx950)
Without --tag: the newest tag that has both files.

Per kernel: average duration, PMC bytes per launch, achieved GB/s and fraction of the 8 TB/s
HBM peak, and -- where the kernel has a per-point algorithmic byte count (below) -- the
algorithmic GB/s and the over-fetch ratio PMC / algorithmic.  For the O(N*M) NN filter:
algorithmic TFLOP/s = 8 flop per (query, model) pair / average duration,
against the 2.5 PF dense f16 MFMA peak of the unit it runs on, and the executed MFMA rate
(32 flop per pair: v_mfma_f32_32x32x16_f16, K = 16) as the matrix-pipe utilisation.

Algorithmic bytes per scene point (fp64 SoA clouds):
  shifted_moments_kernel / gather_moments_kernel: idx 4 + m4[idx] 32 + p 24 + write Y 24 = 84
  centred_moments_kernel: p 24 + Y 24 = 48
  transform_err_kernel (icp_run over a scene in the bundle filter's slot order, the C4 default):
    p 24 + Y 24 + write p 24 + the next search's 64 B slot record + seed16 4 = 140 (no fp32 copy;
    captures up to r03z ran the 92 B form: p 24 + Y 24 + write p 24 + p32 16 + seed16 4)
  NN filter: SURVEY §8d compulsory 12 N + 12 M + 4 N (fp32 xyz in, int32 index out)
From profiles/r04x on (every C4 search the seeded grid search, which writes Y; no bundle record):
  shifted_moments_kernel: p 24 + Y 24 = 48 (the search wrote Y: no index, no gather)
  transform_err_kernel: p 24 + Y 24 + write p 24 + the next search's seed distance 8 = 80
Round 5 (the canonical schedule: one fused grid iteration per seeded iteration):
  canon_moments_kernel (the first iteration's moments; the search wrote Y): p 24 + Y 24 = 48
  canon_transform_kernel (the run's last transform): p 24 + Y 24 + write p 24 + seed distance 8 = 80
  gather_aos_kernel (set_scene into slot order): order 4 + AoS point 24 + write p 24 + fp32 copy 16 = 68
  nn_grid_iter_kernel (GRID_KERNELS): per query p in/out 48 + previous Y 24 + Y out 24 + index
    in/out 8 + the winner's 32-byte grid record = 136; per model point its fp32 grid record 16 +
    cell table 2 = 18
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(ROOT, "profiles")
sys.path.insert(0, os.path.join(ROOT, "tools"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense ~2.5 PF
NN_KERNELS = ("nn_mfma16r_kernel<8>", "nn_mfma16r_kernel<4>", "nn_mfma16_kernel", "nn_mfma16_kernel<seeded>")
BYTES_PER_POINT = {"shifted_moments_kernel": 84, "gather_moments_kernel": 84, "centred_moments_kernel": 48,
                   "transform_err_kernel": 140, "canon_moments_kernel": 48, "canon_transform_kernel": 80,
                   "gather_aos_kernel": 68}


def bytes_per_point(kernel, tag):
    """BYTES_PER_POINT, with the form of the kernels the capture ran: from r04x the grid search's
    (moments streaming Y: 48 B, transform writing the seed distance: 80 B); the slot-record
    transform (140 B) from r03ac; the fp32-copy transform (92 B) before it."""
    if _tag_key(tag) >= _tag_key("r04x") and kernel in ("shifted_moments_kernel", "transform_err_kernel"):
        return {"shifted_moments_kernel": 48, "transform_err_kernel": 80}[kernel]
    if kernel == "transform_err_kernel" and _tag_key(tag) < _tag_key("r03ac"):
        return 92
    return BYTES_PER_POINT[kernel]


def _tag_key(tag):
    """r01t < r01ei < r02a: round number, then suffix length, then suffix."""
    import re
    m = re.match(r"r(\d+)([a-z]*)", tag)
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, tag)


def newest_tag():
    tags = []
    for f in glob.glob(os.path.join(PROFILES, "*_pmc_traffic.json")):
        tag = os.path.basename(f)[: -len("_pmc_traffic.json")]
        if os.path.exists(os.path.join(PROFILES, f"{tag}_bench_kernel_stats.csv")):
            tags.append(tag)
    return max(tags, key=_tag_key) if tags else None


def kernel_times(path):
    from pmc_summary import short
    out = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Name"])
        out[k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) * 1e-6}
    return out


def roofline(tag=None, n=1 << 20, world=1):
    tag = tag or newest_tag()
    if tag is None:
        return None
    times = kernel_times(os.path.join(PROFILES, f"{tag}_bench_kernel_stats.csv"))
    pmc = json.load(open(os.path.join(PROFILES, f"{tag}_pmc_traffic.json")))["kernels"]
    n_local = (n + world - 1) // world
    out = {"tag": tag, "n_model": n, "n_scene_local": n_local, "kernels": {}}
    for k, t in sorted(times.items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["calls"]):
        row = {"calls": t["calls"], "avg_ms": t["avg_ms"]}
        p = pmc.get(k)
        if p and t["avg_ms"] > 0:
            row["pmc_bytes"] = p["traffic_bytes_per_launch"]
            row["pmc_gbps"] = p["traffic_bytes_per_launch"] / (t["avg_ms"] * 1e-3) / 1e9
            row["pmc_hbm_frac"] = row["pmc_gbps"] / HBM_PEAK_GBS
        if k in BYTES_PER_POINT:
            b = bytes_per_point(k, tag) * n_local
            row["algorithmic_bytes"] = b
            row["algorithmic_gbps"] = b / (t["avg_ms"] * 1e-3) / 1e9
            row["hbm_frac"] = row["algorithmic_gbps"] / HBM_PEAK_GBS
            if "pmc_bytes" in row:
                row["over_fetch"] = row["pmc_bytes"] / b
        if k in NN_KERNELS:
            pairs = float(n_local) * n
            row["algorithmic_tflops"] = 8.0 * pairs / (t["avg_ms"] * 1e-3) / 1e12
            row["frac_of_f16_mfma_peak"] = row["algorithmic_tflops"] / F16_MFMA_PEAK_TFLOPS
            row["executed_mfma_tflops"] = 32.0 * pairs / (t["avg_ms"] * 1e-3) / 1e12
            row["mfma_pipe_util"] = row["executed_mfma_tflops"] / F16_MFMA_PEAK_TFLOPS
            cb = 16.0 * n_local + 12.0 * n
            row["compulsory_bytes"] = cb
            row["compulsory_gbps"] = cb / (t["avg_ms"] * 1e-3) / 1e9
        out["kernels"][k] = row
    return out


# ---- the other captures: C3's one-launch registration, the grid variant's resolve ----------
# profiles/<tag>_c3_kernel_stats.csv + <tag>_c3_pmc_traffic.json (+ <tag>_c3_stamps.stamps): rocprofv3
# kernel trace and FETCH_SIZE / WRITE_SIZE passes of `tools/configs_probe.py --configs C3_horse
# --variants auto --reps 1` (BASELINE config C3: horse_ref vs horse_tr1, 50 iterations, one launch
# of icp_persistent_mid_kernel per registration), and its ICP_PERSIST_STAMPS=1 phase timers.
# profiles/<tag>_grid_kernel_stats.csv + <tag>_grid_pmc_traffic.json: the same of `bench.py
# --variant grid` at C4 (nn_grid_resolve_kernel: the seeded exact grid search of every query).
C3_KERNEL = "icp_persistent_mid_kernel"
C3_ITERATIONS = 50
# the grid capture's kernel and its algorithmic bytes (per query, per model point): the seeded
# kernel (round 4: fp64 query 24 B + seed distance 8 + index in 4 / out 4 + correspondence out 24;
# 32-byte grid record + cell table 2) or, in captures before it, the generic resolver's all-mode
# (query 24 + index in/out; 32-byte record) -- its JSON keyed without the template argument
# round 6's nn_grid_iter2_kernel does the same work per launch (the pending transform, the exact
# search of every query, the moments): the same algorithmic bytes, so its fraction compares with
# round 5's kernel directly (it moves less: a certified query reads no model point and writes no
# correspondence, and reads / writes its 16-byte certificate state instead)
GRID_KERNELS = {"nn_grid_iter2_kernel": (136.0, 18.0), "nn_grid_iter_kernel": (136.0, 18.0),
                "nn_grid_seeded_kernel": (64.0, 34.0), "nn_grid_resolve_kernel<4>": (28.0, 32.0)}
GRID_KERNEL = "nn_grid_iter2_kernel"


def grid_kernel_keys(times, pmc):
    """(kernel name in the trace, its key in the PMC JSON, bytes per query, bytes per model point)"""
    for k, (bq, bm) in GRID_KERNELS.items():
        if k in times:
            return k, (k if k in pmc else k.split("<")[0]), bq, bm
    raise KeyError(f"none of {list(GRID_KERNELS)} in the kernel trace")
# workgroup 0's phase timers of the one-launch kernels (icp_iter.hip persist_stamp tags): time
# accumulated into the tag that ENDS each interval
STAMP_PHASES = {0: "iteration turnaround", 1: "nn search", 2: "local sums + publish", 3: "grid barrier wait",
                4: "fold of the published rows", 5: "horn solve + commit", 6: "transform + residual",
                7: "last residual exchange"}


def newest_config_tag(cfg):
    tags = []
    for f in glob.glob(os.path.join(PROFILES, f"*_{cfg}_pmc_traffic.json")):
        tag = os.path.basename(f)[: -len(f"_{cfg}_pmc_traffic.json")]
        if os.path.exists(os.path.join(PROFILES, f"{tag}_{cfg}_kernel_stats.csv")):
            tags.append(tag)
    return max(tags, key=_tag_key) if tags else None


def stamp_phases(path):
    """Mean per-registration time of each phase (us) over the [persist] lines of a stamps log."""
    import re
    runs = []
    for line in open(path):
        if not line.startswith("[persist] grid"):
            continue
        body = line.split("(calls):", 1)[1].split("|", 1)[0]
        ph = {}
        for tag, us, calls in re.findall(r"(\d+):([\d.]+)\((\d+)\)", body):
            if int(calls) > 0 and int(tag) in STAMP_PHASES:
                ph[STAMP_PHASES[int(tag)]] = float(us)
        runs.append(ph)
    if not runs:
        return None
    keys = runs[0].keys()
    return {k: sum(r.get(k, 0.0) for r in runs) / len(runs) for k in keys}


def config_roofline(cfg, tag=None, n=1 << 20):
    """cfg "c3": bytes per registration of the one-launch kernel, its rate and HBM fraction, bytes
    per iteration, the phase split; cfg "grid": the seeded grid search at C4 (n queries, n model
    points) against its algorithmic bytes (GRID_KERNELS)."""
    tag = tag or newest_config_tag(cfg)
    if tag is None:
        return None
    times = kernel_times(os.path.join(PROFILES, f"{tag}_{cfg}_kernel_stats.csv"))
    pmc = json.load(open(os.path.join(PROFILES, f"{tag}_{cfg}_pmc_traffic.json")))["kernels"]
    if cfg == "c3":
        k = kp = C3_KERNEL
    else:
        k, kp, bq, bm = grid_kernel_keys(times, pmc)
    t, p = times[k], pmc[kp]
    sec = t["avg_ms"] * 1e-3
    b = p["traffic_bytes_per_launch"]
    out = {"tag": tag, "kernel": k, "source": f"profiles/{tag}_{cfg}_kernel_stats.csv + profiles/{tag}_{cfg}_pmc_traffic.json",
           "launches": t["calls"], "avg_ms": t["avg_ms"], "pmc_bytes_per_launch": b, "pmc_gbps": b / sec / 1e9,
           "pmc_hbm_frac": b / sec / 1e9 / HBM_PEAK_GBS, "fetch_bytes": p.get("fetch_bytes_per_launch"),
           "write_bytes": p.get("write_bytes_per_launch")}
    if cfg == "c3":
        out["iterations_per_launch"] = C3_ITERATIONS
        out["pmc_bytes_per_iteration"] = b / C3_ITERATIONS
        sp = os.path.join(PROFILES, f"{tag}_c3_stamps.stamps")
        if os.path.exists(sp):
            out["phases_us_per_registration"] = stamp_phases(sp)
            out["phases_source"] = f"profiles/{tag}_c3_stamps.stamps (ICP_PERSIST_STAMPS=1, workgroup 0)"
    else:
        alg = bq * n + bm * n
        out["algorithmic_bytes"] = alg
        out["algorithmic_gbps"] = alg / sec / 1e9
        out["hbm_frac"] = out["algorithmic_gbps"] / HBM_PEAK_GBS
        out["over_fetch"] = b / alg
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--config", choices=["c4", "C3", "c3", "grid"], default="c4",
                    help="c4: the bench's kernels; C3: the one-launch C3 registration; grid: the grid variant")
    a = ap.parse_args()
    if a.config.lower() != "c4":
        r = config_roofline(a.config.lower(), a.tag, a.n)
        if r is None:
            sys.exit(f"no profiles/<tag>_{a.config.lower()}_pmc_traffic.json + _kernel_stats.csv pair found")
        print(json.dumps(r, indent=1))
        return
    r = roofline(a.tag, a.n, a.world)
    if r is None:
        sys.exit("no profiles/<tag>_pmc_traffic.json + <tag>_bench_kernel_stats.csv pair found")
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
