#!/usr/bin/env python3
"""bench.py — ICP iterations/s on MI355X (BASELINE.json metric, config C4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--points N] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[3]): synthetic 2^20-point model uniform in
[-1,1]^3 (mt19937_64 seed 42), scene = R(5 deg about (1,2,3)) model + (0.05,-0.03,0.02),
fixed iterations (threshold disabled).  One step = one complete registration of 30 ICP
iterations (SURVEY §8d's clock, from the model's preparation on): icp_set_model_device (every
model image built on the device), icp_set_scene_device, icp_run(30) -- each iteration the exact
NN of every scene point against the whole model, centroids, cross-covariance, Horn solve,
transform + residual.  value = steps x 30 iterations / wall time.  The clouds are device arrays
resident in HBM before the timed region starts (no PCIe inside `value`; the PCIe-inclusive
registration from host arrays is reported beside it, `registration`), and `steady_state` gives
the rate of the seeded iterations alone.  Multi-GPU: the scene is sharded over ranks (model
replicated), sums are all-reduced with RCCL inside libicp_hip.so; total work is fixed =>
"strong".

Timed region: K registrations, bracketed by a barrier + device synchronisation on both sides;
ms_per_step = max over ranks.
roofline: the level-1 O(N*M) NN filter kernel, timed with HIP events on the engine's stream.
achieved = ALGORITHMIC flop (8 per (query, model) pair, this rank's shard x the
whole model) / average launch time, against the peak of the unit the kernel runs on: the 2.5 PF
dense f16 MFMA peak for the default f16 filter, 157.3 TF for the fp32 filters.  The executed MFMA
rate (32 flop per pair, K = 16) is reported beside it as the matrix-pipe utilisation.  traffic:
HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/*_pmc_traffic.json) when
the run matches its workload; nn_hbm: the metric's "NN achieved HBM GB/s" (PMC bytes and the
compulsory bytes of §8d over the live launch time).  streaming: the bandwidth-bound kernels of
the iteration from the committed profiles (tools/roofline.py recomputes every figure).
cpu_baseline: the oracle (C restatement of src/cpu.cc, 1 core) on rank 0: NN on a
4096-query sample against the full model, scaled by N/4096, + the O(N) steps in full.
N > 1: rank 0 also reports every rank's filter time and its measured per-iteration all-reduce
latency (HIP events around the collective on the engine stream).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

import icp_amd  # noqa: E402
import roofline as RF  # noqa: E402

GRID_SEEDED_KERNEL = "nn_grid_seeded_kernel"  # (tools/roofline.py GRID_KERNELS: its algorithmic bytes)
# the fused grid iteration (transform + seeded search + moments, one launch per seeded iteration:
# icp_run's canonical schedule); ICP_GRID_ITER=0 runs the separate kernels
GRID_ITER_KERNEL = "nn_grid_iter2_kernel"  # (round 6: the exclusion certificate + packed walkers)
GRID_ITER_KERNEL_R5 = "nn_grid_iter_kernel"  # (ICP_ITER_V2=0: round 5's two-lane kernel, every query walks)


def grid_kernel():
    if os.environ.get("ICP_GRID_ITER") == "0":
        return GRID_SEEDED_KERNEL
    return GRID_ITER_KERNEL_R5 if os.environ.get("ICP_ITER_V2") == "0" else GRID_ITER_KERNEL


def path_description(st):
    """What the timed registrations ran, from one registration's counters (icp_stats): the
    searches by kind, the fused iterations' certified / walked queries."""
    g, b = st["run_grid_searches"], st["run_bundle_searches"]
    cert, walk = st["run_certified"], st["run_walked"]
    parts = []
    if g:
        parts.append(f"{g} exact fp64 grid searches (fp32 screen, candidates decided in fp64: the first "
                     "from cell seeds, the seeded ones the fused grid iteration "
                     f"{grid_kernel()}" + (f", {cert / max(cert + walk, 1):.0%} of its queries kept their "
                                           "correspondence by the exclusion certificate without a walk"
                                           if cert + walk else "") + ")")
    if b:
        parts.append(f"{b} searches through the f16 hi/lo-split MFMA bundle bound + pair filter (fp32 "
                     "accumulate) with the fp64 certificate")
    return ("; ".join(parts) or "no search") + "; fp64 transform and reductions"

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = f32 MFMA peak
PEAK_F16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/FP16 MFMA ~2.5 PF dense
FLOP_PER_PAIR = 8          # SURVEY.md §8d (algorithmic: 3 sub + 1 mul + 2 fma)
MFMA16_FLOP_PER_PAIR = 32  # executed: v_mfma_f32_32x32x16_f16 = 2*32*32*16 flop per 1024 pairs
REF_OPTI_GPU_LOOP_FPS = 9.36368  # reference README.md:108 (GTX 1050, cow_ref/cow_tr1)
# the reference's published google-benchmark times, ms per iteration (README.md:95-108;
# GTX 1050 / i7-4790 1 thread, cow_ref vs cow_tr1; *_loop = one complete registration)
REF_README_MS = {
    "cpu_closest_matrix": 8726, "naive_gpu_closest_matrix": 2935, "opti_gpu_closest_matrix": 7.46,
    "cpu_find_alignment": 14.9, "gpu_find_alignment": 5.52, "cpu_compute_centroid": 1.33,
    "gpu_compute_centroid": 2.38, "cpu_err_compute": 8.44, "gpu_err_compute": 1.16,
    "cpu_err_compute_alignment": 8.54, "gpu_err_compute_alignment": 1.75, "cpu_loop": 61276,
    "naive_gpu_loop": 18240, "opti_gpu_loop": 107,
}


def progress(msg):
    """A line on stderr per phase (rank 0): a long multi-rank run shows it is alive."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def pmc_traffic(kernel, cfg=None):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (written by tools/pmc_summary.py from separate FETCH_SIZE and WRITE_SIZE passes, FETCH_SIZE
    doubled per the gfx950 correction): profiles/<tag>_pmc_traffic.json for this bench at C4 on
    one GPU, profiles/<tag>_<cfg>_pmc_traffic.json for another workload (cfg "c5shard": rank 0's
    shard of the 8-way C5, tools/gpu_round.sh c5pmc)."""
    import glob
    from roofline import _tag_key
    paths = glob.glob(os.path.join(ROOT, "profiles", f"*_{cfg}_pmc_traffic.json" if cfg else "*_pmc_traffic.json"))
    if not cfg:  # (this bench's own captures: <tag>_pmc_traffic.json, no workload label)
        paths = [f for f in paths if os.path.basename(f).count("_") == 2]
    for path in sorted(paths, key=lambda f: _tag_key(os.path.basename(f).split("_")[0]), reverse=True):
        try:
            k = json.load(open(path))["kernels"].get(kernel)
        except (OSError, ValueError, KeyError):
            continue
        if k:
            return k["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(m, p, sample=4096, seed=0):
    """Oracle (src/cpu.cc restatement) on this host: one core (the reference's own CPU path is
    single-threaded), and all the cores this job may use (OMP_NUM_THREADS, else nproc; the
    oracle's closest_range calls release the GIL, so a thread pool runs them in parallel)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O
    from concurrent.futures import ThreadPoolExecutor
    O.lib()
    n = p.shape[0]
    rng = np.random.default_rng(seed)
    sel = np.sort(rng.choice(n, size=min(sample, n), replace=False))
    t0 = time.perf_counter()
    y_s, _ = O.closest(p[sel], m)
    t_nn = (time.perf_counter() - t0) * n / sel.size
    # O(N) steps in full on a correspondence set of the right size
    y = np.empty_like(p)
    y[:] = m[np.arange(n) % m.shape[0]]
    t0 = time.perf_counter()
    al = O.find_alignment(p, y)
    O.err_compute(p, y, al.s, al.R, al.t)
    t_lin = time.perf_counter() - t0
    per_iter = t_nn + t_lin
    out = {"value": 1.0 / per_iter, "unit": "ICP iterations/s", "cores": 1, "kind": "port",
           "sample": f"NN of {sel.size} of {n} queries vs all {m.shape[0]} model points "
                     f"({t_nn * sel.size / n:.1f} s, scaled x{n / sel.size:.0f}) + full O(N) "
                     f"alignment/transform ({t_lin:.3f} s)",
           "seconds_per_iteration": per_iter, "cpu_model": _cpu_model()}
    # all cores: the same per-query NN over a proportionally larger sample, split in chunks
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    if threads > 1:
        sel_t = np.sort(rng.choice(n, size=min(sample * threads, n), replace=False))
        pt = np.ascontiguousarray(p[sel_t])
        bounds = np.linspace(0, pt.shape[0], threads + 1).astype(int)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda k: O.closest(pt, m, O.NN_SQUARED, int(bounds[k]), int(bounds[k + 1])),
                        range(threads)))
        t_nn_t = (time.perf_counter() - t0) * n / sel_t.size
        per_t = t_nn_t + t_lin  # the O(N) steps stay single-threaded (0.1% of an iteration)
        out["all_cores"] = {"value": 1.0 / per_t, "cores": threads, "seconds_per_iteration": per_t,
                            "sample": f"NN of {sel_t.size} queries on {threads} threads "
                                      f"({t_nn_t * sel_t.size / n:.1f} s, scaled x{n / sel_t.size:.0f})"}
    return out


def rank_record(rank, info, filter_ms, allreduce_ms, n_local, iterations, ms_per_step=None, reg=None):
    """One rank's entry of the line's per_rank: its own ms per iteration, its level-1 filter time
    (HIP events on the engine stream), the rest of its iteration (tail_ms: the other launches and
    the all-reduce), its per-iteration all-reduce latency, its registration cost (set_model ms,
    whole-registration ms), and what it ran on -- its RCCL communicator's ncclCommCount /
    ncclCommUserRank (null / its own rank without RCCL) and the PCI bus id of its device
    (icp_get_comm_info)."""
    return {"rank": rank, "ms_per_step": ms_per_step, "filter_ms": filter_ms,
            "tail_ms": (ms_per_step - filter_ms) if ms_per_step is not None and filter_ms else None,
            "allreduce_ms_per_iter": allreduce_ms,
            "set_model_ms": reg["set_model_ms"] if reg else None,
            "registration_ms": reg["registration_ms"] if reg else None,
            "n_scene_local": n_local, "iterations": iterations, "comm_count": info["comm_count"],
            "comm_rank": info["comm_rank"], "pci_bus_id": info["pci_bus_id"]}


def check_devices(per_rank, world, rccl):
    """None if the ranks are what the line claims, else why not.  With RCCL every rank must
    sit in one communicator of `world` ranks, at its own rank, on its own GPU (N distinct PCI
    bus ids); without RCCL (1 rank, or the gloo rehearsal of several ranks on one GPU) only the
    ranks themselves are checked."""
    ranks = sorted(r["rank"] for r in per_rank)
    if ranks != list(range(world)):
        return f"per_rank holds ranks {ranks}, expected 0..{world - 1}"
    if not rccl:
        return None
    bad = [r["rank"] for r in per_rank if r["comm_count"] != world or r["comm_rank"] != r["rank"]]
    if bad:
        return f"ranks {bad} are not rank r of a {world}-rank RCCL communicator"
    buses = [r["pci_bus_id"] for r in per_rank]
    if len(set(buses)) != world:
        return f"{world} RCCL ranks on {len(set(buses))} distinct GPUs ({sorted(buses)})"
    return None


def _cow_paths():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import datasets
    return datasets.path("cow_ref"), datasets.path("cow_tr1")


BUNDLE_COUNT_STEPS = 3
REGISTRATION_ITERS = 30  # BASELINE.json configs[3] / [4]: 30 iterations
STEADY_ITERS = 60        # the steady-state line: seeded iterations of one continued registration


def bundle_v1():
    """ICP_BUNDLE_KERNEL=1 selects the v1 bundle filter (nn_bundle_kernel); v2 (nn_bundle2_kernel,
    with bundle_prep_kernel + bundle_group_kernel before it) is the default."""
    return os.environ.get("ICP_BUNDLE_KERNEL") == "1"


def bundle_roofline(n_local, n_model, t_kernel, work, v1=False):
    """The bundle filter against the f16 MFMA peak on the work it EXECUTES, counted on the device
    (icp_set_bundle_counters): the stream's group-bound tests (one v_mfma_f32_32x32x16_f16 =
    2*32*32*16 flop per 32-bundle block per workgroup: the workgroup's 32 query groups x 32
    bundles), the per-query bound tests on the groups a fired block fired for (32 queries x 32
    bundles each) and the pair tests (32 queries x 32 points each); v1 also re-issued each fired
    block's stream test.  The N x M pairs the search decides are listed beside it as
    effective_pairs_per_s; SURVEY §8d's 8 flop per pair over them is no roofline here (most pairs
    are excluded by the bounds, not evaluated)."""
    stream = work["stream_mfma"]
    fired = work["block_triggers"]
    reissued = fired if v1 else 0.0
    fine = work["group_tests"]
    pair = work["pair_tests"]
    executed = 32768.0 * (stream + reissued + fine + pair)
    ach = executed / t_kernel / 1e12
    return {"bound": "mfma", "compute_unit": "v_mfma_f32_32x32x16_f16: bound |x-c|^2-(D+r)^2 of each 32-query group "
                                             "(then of each query) against each 32-point kd bundle (hi/lo split, "
                                             "16 products), then the f16 pair test of the bundles it cannot exclude",
            "achieved": ach, "peak": PEAK_F16_MFMA_TFLOPS, "frac": ach / PEAK_F16_MFMA_TFLOPS,
            "flop_per_launch": executed,
            "flop_definition": "executed f16 MFMA work (2*32*32*16 flop per instruction), per launch: "
                               f"{stream:.0f} stream bound tests + {reissued:.0f} re-issued on fired blocks + "
                               f"{fine:.0f} per-query bound tests + {pair:.0f} pair tests (device counters over "
                               f"{BUNDLE_COUNT_STEPS} seeded iterations)",
            "wave_task_phases_us": work.get("us_per_wave_task"),
            "work_per_launch": {"stream_mfma": stream, "fired_blocks": fired, "reissued_stream_mfma": reissued,
                                "group_tests": fine, "pair_tests": pair, "pairs_evaluated": 1024.0 * pair,
                                "pair_share_of_n_m": 1024.0 * pair / (n_local * n_model)},
            "effective_pairs_per_s": n_local * n_model / t_kernel,
            "pairs_per_s": n_local * n_model / t_kernel}


def grid_roofline(n_local, n_model, avg_ms, traffic, traffic_src, explicit_variant):
    """The grid iteration's dominant kernel (nn_grid_iter_kernel: the pending transform, the seeded
    search of every query and the moments' leaves in one launch; nn_grid_seeded_kernel with
    ICP_GRID_ITER=0) against HBM.  Algorithmic bytes per launch (tools/roofline.py GRID_KERNELS):
    fused -- per query its fp64 position in and out (48 B), previous and new correspondence (48 B),
    index in and out (8 B) and the winner's 32-byte grid record; per model point its 16-byte fp32
    grid record and ~2 B of the cell table, once.  Seeded alone -- 64 B per query, 34 B per model
    point."""
    kern = grid_kernel()
    bq, bm = RF.GRID_KERNELS[kern]
    gbytes = bq * n_local + bm * n_model
    t = avg_ms * 1e-3
    ach = gbytes / t / 1e9 if t > 0 else 0.0
    what = {GRID_ITER_KERNEL: "fused grid iteration: transform + exclusion certificate + packed walks of the rest "
                              "+ moments, every query",
            GRID_ITER_KERNEL_R5: "fused grid iteration: transform + seeded search + moments, every query"}.get(
        kern, "seeded, every query")
    return {"bound": "hbm", "kernel": f"{kern} ({what})",
            "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0,
            "traffic": traffic, "traffic_unit": "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src, "avg_launch_ms": avg_ms, "bytes_per_launch": gbytes,
            "bytes_definition": f"algorithmic: {bq:.0f} B per query + {bm:.0f} B per model point, once "
                                "(tools/roofline.py GRID_KERNELS)",
            "path": "ICP_NN_VARIANT_GRID" if explicit_variant else
                    "AUTO: icp_run's policy (seeded iterations once the scene is near the model)",
            "note": "latency-bound: the walkers' dependent loads (cell table, points, candidate records) set each "
                    "wave's time (DESIGN §3.8)"}


def full_nxm_rate(device, m, p, steps=5, warmup=2):
    """The full N x M f16 filter (ICP_NN_VARIANT_MFMA16, nn_mfma16r_kernel<8>) on the same C4
    iterations, for comparison with the bundle filter: same results bit for bit."""
    with icp_amd.Context(device) as ctx:
        ctx.set_nn_variant(icp_amd.VARIANT_MFMA16)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(warmup, -1.0)
        ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.run(steps, -1.0)
        dt = time.perf_counter() - t0
        st = ctx.stats()
    t = st["nn_ms"] / max(st["nn_launches"], 1) * 1e-3
    pairs = float(p.shape[0]) * m.shape[0]
    ach = FLOP_PER_PAIR * pairs / t / 1e12
    return {"kernel": "nn_mfma16r_kernel<8>", "iterations_per_s": steps / dt, "avg_launch_ms": t * 1e3,
            "achieved": ach, "peak": PEAK_F16_MFMA_TFLOPS, "frac": ach / PEAK_F16_MFMA_TFLOPS,
            "flop_definition": "algorithmic: 8 flop per (query, model) pair over all N x M pairs",
            "executed_tflops": MFMA16_FLOP_PER_PAIR * pairs / t / 1e12, "pairs_per_s": pairs / t}


def reference_cases_gpu(min_time=0.3):
    """The reference's 8 GPU benchmark cases (src/bench.cc:391-445) through
    iterative-closest-point_amd/build/icp-bench, on the bundled cow pair."""
    import subprocess
    ref, scene = _cow_paths()
    exe = os.path.join(ROOT, "iterative-closest-point_amd", "build", "icp-bench")
    r = subprocess.run([exe, "--ref", ref, "--scene", scene, "--min-time", str(min_time), "--json"],
                       capture_output=True, text=True, timeout=600, check=True)
    cases = json.loads(r.stdout.strip().splitlines()[-1])["cases"]
    # the reference's opti_gpu_loop re-uploads the model on every frame (compute.cu:160): the
    # same case with icp_set_model inside each registration
    r = subprocess.run([exe, "--ref", ref, "--scene", scene, "--min-time", str(min_time), "--json", "--cold",
                        "--only", "opti_gpu_loop_cold"], capture_output=True, text=True, timeout=600, check=True)
    cases.update(json.loads(r.stdout.strip().splitlines()[-1])["cases"])
    REF_README_MS.setdefault("opti_gpu_loop_cold", REF_README_MS["opti_gpu_loop"])
    return {k: {"ms": v["ms"], "frame_rate": v["frame_rate"], "reference_ms": REF_README_MS.get(k),
                "speedup_vs_reference": (REF_README_MS[k] / v["ms"]) if k in REF_README_MS else None}
            for k, v in cases.items()}


def reference_cases_cpu(reps=3):
    """The reference's 6 CPU cases on this host with the oracle (the C restatement of
    src/cpu.cc, 1 core); cpu_compute_centroid is numpy (Eigen's rowwise mean + colwise -)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O
    m, p = (O.load_matrix(x) for x in _cow_paths())
    y, _ = O.closest(p, m, O.NN_CPU_SQRT)
    al = O.find_alignment(p, y)
    R = np.array(al.R).reshape(3, 3)

    def t(f, n=reps):
        f()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        return (time.perf_counter() - t0) * 1e3 / n

    def centroid():
        for a in (p, y):
            _ = a - a.mean(axis=0)

    ms = {
        "cpu_closest_matrix": t(lambda: O.closest(p, m, O.NN_CPU_SQRT), 1),
        "cpu_find_alignment": t(lambda: O.find_alignment(p, y)),
        "cpu_compute_centroid": t(centroid),
        "cpu_err_compute": t(lambda: O.err_compute(p, y, al.s, R, al.t)),
        "cpu_err_compute_alignment": t(lambda: O.err_compute_alignment(p, y, al.s, R, al.t)),
        "cpu_loop": t(lambda: O.icp(m, p, 20, 1e-5, O.NN_CPU_SQRT), 1),
    }
    return {k: {"ms": v, "reference_ms": REF_README_MS[k], "speedup_vs_reference": REF_README_MS[k] / v}
            for k, v in ms.items()}


def grid_nn_rate(device, m, p, steps, warmup=3):
    """the same C4 iterations with ICP_NN_VARIANT_GRID (exact fp64 search
    on the model grid, no brute-force filter).  Reported beside the headline, not as it."""
    with icp_amd.Context(device) as ctx:
        ctx.set_nn_variant(icp_amd.VARIANT_GRID)
        ctx.set_model(m)
        ctx.set_scene(p)
        ctx.run(warmup, -1.0)
        ctx.reset_stats()
        t0 = time.perf_counter()
        _, errs = ctx.run(steps, -1.0)
        dt = time.perf_counter() - t0
        st = ctx.stats()
    return {"iterations_per_s": steps / dt, "ms_per_step": dt * 1e3 / steps,
            "nn_kernel_ms": st["nn_ms"] / max(st["nn_launches"], 1), "brute_force_fallbacks": st["grid_fallback"],
            "final_err": float(errs[-1]), "kernel": grid_kernel(),
            "roofline": grid_roofline(p.shape[0], m.shape[0], st["nn_ms"] / max(st["nn_launches"], 1),
                                      *pmc_traffic(grid_kernel()), True)}


def baseline_configs(device, reps=3):
    """BASELINE.json configs C2 (bun000 vs bun045, allow_unequal) and C3 (horse_ref vs horse_tr1):
    complete 50-iteration registrations (reference semantics, threshold 1e-5; neither converges
    within 50) on this GPU with the default path -- one launch per registration
    (icp_persistent_mid_kernel: culled exact fp64 NN) -- and beside it the launch loop with the
    brute-force f16 MFMA filter and the exact grid variant (the same trajectory bit for bit)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import datasets

    def registration(m, p, unequal, variant, mode=icp_amd.RUN_AUTO):
        with icp_amd.Context(device) as ctx:
            ctx.set_nn_variant(variant)
            ctx.set_run_mode(mode)
            ctx.set_allow_unequal(unequal)
            ctx.set_model(m)
            ctx.set_scene(p)
            ctx.run(50)  # warm
            ctx.reset_stats()
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.set_scene(p)
                res, errs = ctx.run(50)
            return res, errs, (time.perf_counter() - t0) / reps, ctx.stats()

    out = {}
    for name, (ref, scene, unequal) in {"C2_bun000_bun045": ("bun000", "bun045", True),
                                        "C3_horse_ref_tr1": ("horse_ref", "horse_tr1", False)}.items():
        m = icp_amd.load_matrix(datasets.path(ref))
        p = icp_amd.load_matrix(datasets.path(scene))
        res, errs, dt, st = registration(m, p, unequal, icp_amd.VARIANT_AUTO)
        lres, lerrs, ldt, lst = registration(m, p, unequal, icp_amd.VARIANT_AUTO, icp_amd.RUN_LAUNCHES)
        gres, gerrs, gdt, _ = registration(m, p, unequal, icp_amd.VARIANT_GRID)
        out[name] = {"n_model": int(m.shape[0]), "n_scene": int(p.shape[0]), "iterations": res.iterations,
                     "ms_per_registration": dt * 1e3, "iterations_per_s": res.iterations / dt,
                     "path": "one launch per registration" if st["persistent_runs"] else "launch loop",
                     "final_err": float(errs[res.iterations - 1]),
                     "launch_loop": {"iterations_per_s": lres.iterations / ldt, "ms_per_registration": ldt * 1e3,
                                     "nn_filter_ms": lst["nn_ms"] / max(lst["nn_launches"], 1),
                                     "same_trajectory": bool(np.array_equal(lerrs, errs))},
                     "grid_variant": {"iterations_per_s": gres.iterations / gdt, "ms_per_registration": gdt * 1e3,
                                      "same_trajectory": bool(np.array_equal(gerrs, errs))}}
    rf = committed_config_roofline("c3")
    if rf is not None:
        # the one-launch C3 registration's HBM bytes and rate from its committed rocprofv3 capture
        # (tools/roofline.py --config C3): a measured profile of this same configuration, not of
        # this run
        out["C3_horse_ref_tr1"]["hbm"] = rf
    return out


def committed_config_roofline(cfg):
    """tools/roofline.config_roofline over the newest committed profiles/<tag>_<cfg>_* pair
    (None when there is none; an error string when it does not parse)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import roofline as RF
        return RF.config_roofline(cfg)
    except Exception as e:  # a malformed profile must not break the bench line
        return {"error": str(e)}


def csv_io(m):
    """load.cc:3-97 at C4 size: write the model (ostream %g rows) and load it back
    (sscanf %lf rows) with the product's parallel exact parser / formatter."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "cloud.txt")
        t0 = time.perf_counter()
        icp_amd.write_matrix(f, m)
        tw = time.perf_counter() - t0
        size = os.path.getsize(f)
        t0 = time.perf_counter()
        back = icp_amd.load_matrix(f)
        tl = time.perf_counter() - t0
    return {"rows": int(m.shape[0]), "bytes": size, "write_s": tw, "load_s": tl,
            "load_mb_per_s": size / tl / 1e6, "roundtrip_rows": int(back.shape[0])}


def torch_stream(t):
    """The HIP stream handle of torch's current stream on tensor t's device."""
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def registration(ctx, m, p_local, n_total, iters=30, reps=3, device=None):
    """SURVEY §8d's clock: a whole registration from model upload through the last iteration's
    err -- icp_set_model (host AoS in, every device image built), icp_set_scene, the first
    (unseeded) iteration and the seeded ones.  Each rep re-uploads both clouds (set_model always
    rebuilds), on the caller's context (one-time hipInit / RCCL init excluded, as §8d says).
    The first iteration is timed by a separate run(1) after a fresh set_scene; the seeded ones
    are the rest of the 30-iteration run.  device = (model tensor, scene tensor): the same phases
    from device-resident clouds (icp_set_model_device / icp_set_scene_device: the headline's step)."""
    def set_model():
        if device is None:
            ctx.set_model(m)
        else:
            ctx.set_model_device(device[0].data_ptr(), m.shape[0], stream=torch_stream(device[0]))

    def set_scene():
        if device is None:
            ctx.set_scene(p_local, np_total=n_total)
        else:
            ctx.set_scene_device(device[1].data_ptr(), p_local.shape[0], n_total, stream=torch_stream(device[1]))

    rows = []
    for _ in range(reps):
        t0 = time.perf_counter()
        set_model()
        t1 = time.perf_counter()
        set_scene()
        t2 = time.perf_counter()
        res, _ = ctx.run(iters, -1.0)
        t3 = time.perf_counter()
        set_scene()
        t4 = time.perf_counter()
        ctx.run(1, -1.0)
        t5 = time.perf_counter()
        rows.append((t1 - t0, t2 - t1, t3 - t2, t5 - t4, res.iterations))
    a = np.median(np.array(rows, dtype=np.float64), axis=0)
    set_model, set_scene, run_all, first, its = a
    total = set_model + set_scene + run_all
    return {"iterations": int(its), "reps": reps, "set_model_ms": set_model * 1e3, "set_scene_ms": set_scene * 1e3,
            "first_iteration_ms": first * 1e3,
            "seeded_iteration_ms": (run_all - first) * 1e3 / max(its - 1, 1),
            "run_ms": run_all * 1e3, "registration_ms": total * 1e3,
            "iterations_per_s_inclusive": its / total,
            "set_model_ms_per_rep": [r[0] * 1e3 for r in rows],
            "definition": "median over reps of wall time: set_model (host fp64 AoS -> every device image) + "
                          f"set_scene + icp_run({iters}); first_iteration_ms = run(1) after a fresh set_scene "
                          "(slot order, grid seeds, unseeded search); seeded = the rest of the run per iteration"}


def cow_frame_rate(device, reps=20):
    """Reference headline: opti_gpu_loop frame_rate = complete cow registrations/s."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import datasets
    m = icp_amd.load_matrix(datasets.path("cow_ref"))
    p = icp_amd.load_matrix(datasets.path("cow_tr1"))
    with icp_amd.Context(device) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        res, _ = ctx.run(20)  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.set_scene(p)  # a fresh GPU::ICP per benchmark iteration (bench.cc:70-76)
            res, _ = ctx.run(20)
        dt = (time.perf_counter() - t0) / reps
    return {"frames_per_s": 1.0 / dt, "iterations_per_frame": res.iterations,
            "vs_reference_opti_gpu_loop": (1.0 / dt) / REF_OPTI_GPU_LOOP_FPS}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    # (--points under torchrun: its own parser takes a bare "--n" for an ambiguous prefix of
    # --nnodes / --nproc-per-node and stops)
    ap.add_argument("--points", "--n", dest="n", type=int, default=1 << 20)
    ap.add_argument("--nn", choices=["certified", "fp64"], default="certified")
    ap.add_argument("--variant", choices=["auto", "valu", "mfma", "mfma16", "grid", "bundle"], default="auto")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cow", action="store_true")
    ap.add_argument("--no-cases", action="store_true", help="skip the reference's 14 benchmark cases")
    ap.add_argument("--no-registration", dest="registration", action="store_false",
                    help="skip the registration block (SURVEY §8d: set_model through the last iteration)")
    ap.add_argument("--rccl", action="store_true",
                    help="N=1: route the per-iteration sums through a 1-rank RCCL communicator, as N>1 does")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")  # control plane only; the data path is RCCL in the engine
    import torch
    # one GPU per rank; fewer GPUs than ranks happens only in the gloo rehearsal
    ndev = icp_amd.device_count()
    if ndev > 0 and local >= ndev:
        local = local % ndev

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(local)

    nn_mode = icp_amd.NN_CERTIFIED if args.nn == "certified" else icp_amd.NN_FP64
    if world > 1 and os.environ.get("ICP_BENCH_HOST_REDUCE") == "1":
        # rehearsal of the multi-rank flow where RCCL cannot run (several ranks on one GPU):
        # the engine's sums go through gloo instead; timing and results are otherwise the same
        def host_allreduce(buf):
            t = torch.from_numpy(buf.copy())
            dist.all_reduce(t)
            buf[:] = t.numpy()
        ctx = icp_amd.Context(local, nn_mode, rank, world, host_allreduce=host_allreduce)
    elif world > 1:
        obj = [icp_amd.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx = icp_amd.Context(local, nn_mode, rank, world, obj[0])
    elif args.rccl:
        ctx = icp_amd.Context(local, nn_mode, 0, 1, icp_amd.rccl_unique_id())
    else:
        ctx = icp_amd.Context(local, nn_mode)

    variant = {"auto": icp_amd.VARIANT_AUTO, "valu": icp_amd.VARIANT_VALU, "mfma": icp_amd.VARIANT_MFMA,
               "mfma16": icp_amd.VARIANT_MFMA16, "grid": icp_amd.VARIANT_GRID,
               "bundle": icp_amd.VARIANT_BUNDLE}[args.variant]
    ctx.set_nn_variant(variant)
    m, p = icp_amd.synthetic_pair(args.n, seed=42)
    b, c = icp_amd.shard_range(args.n, rank, world)
    # The clouds resident in HBM before anything is timed (device arrays: torch is plumbing here):
    # a step is ONE complete registration -- icp_set_model_device (every model image: stats, fp32 /
    # f16 images, grid; the bundle images when the policy needs them), icp_set_scene_device (SoA
    # copies, slot order), icp_run(30) -- SURVEY §8d's clock from the model's preparation on,
    # without the PCIe copy (reported beside it: registration_pcie)
    dev = f"cuda:{local}"
    dm = torch.from_numpy(np.ascontiguousarray(m)).to(dev)
    dps = torch.from_numpy(np.ascontiguousarray(p[b:b + c])).to(dev)
    torch.cuda.synchronize(local)

    # (the clouds were written on torch's current stream: the engine's stream waits for it,
    # icp_set_*_device_stream, without a device synchronisation)
    sm = torch_stream(dm)

    def registration_step():
        ctx.set_model_device(dm.data_ptr(), m.shape[0], stream=sm)
        ctx.set_scene_device(dps.data_ptr(), c, args.n, stream=sm)
        return ctx.run(REGISTRATION_ITERS, -1.0)

    progress("model and scene resident")
    for _ in range(args.warmup):
        registration_step()
    progress("warm-up done")
    ctx.reset_stats()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, errs = registration_step()
    barrier_sync()
    dt = time.perf_counter() - t0
    dt_local = dt
    st = ctx.stats()
    # the steady-state rate beside it: the last registration continued (seeded iterations only)
    ctx.run(3, -1.0)
    barrier_sync()
    t1 = time.perf_counter()
    ctx.run(STEADY_ITERS, -1.0)
    barrier_sync()
    dt_ss = time.perf_counter() - t1
    if dist is not None:
        t = torch.tensor([dt, dt_ss], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dt_ss = float(t[0].item()), float(t[1].item())

    # the level-1 filter the engine ran (icp_stats.last_filter), not a guess from the sizes
    level1 = icp_amd.FILTER_NAMES.get(st["last_filter"])
    if level1 in ("valu", "fp64", "one_launch"):
        level1 = None
    nn_avg_ms = st["nn_ms"] / max(st["nn_launches"], 1)
    ar_ms = st["allreduce_ms"] / st["allreduce_calls"] if st["allreduce_calls"] else None
    work = None
    if level1 == "bundle":
        # untimed, after the timed region, on every rank (icp_run all-reduces): the bundle
        # filter's executed work per search from its device counters, over a few more seeded
        # iterations of the same registration
        ctx.set_bundle_counters(True)
        ctx.run(BUNDLE_COUNT_STEPS, -1.0)
        bc = ctx.bundle_counters()
        work = {k: v / BUNDLE_COUNT_STEPS for k, v in bc.items() if not isinstance(v, dict)}
        work["us_per_wave_task"] = bc["us_per_wave_task"]
        ctx.set_bundle_counters(False)
    # SURVEY §8d's clock: whole registrations from the model upload (every rank: icp_run
    # all-reduces), untimed by the headline
    progress("timed iterations done")
    reg = registration(ctx, m, p[b:b + c], args.n, iters=REGISTRATION_ITERS) if args.registration else None
    # the headline step's phases (device-resident clouds), untimed by the headline
    reg_dev = registration(ctx, m, p[b:b + c], args.n, iters=REGISTRATION_ITERS, device=(dm, dps))
    # what a timed step ran: one more registration's counters (the searches by kind, the fused
    # iterations' certified / walked queries), for the line's dtype
    ctx.reset_stats()
    registration_step()
    path_st = ctx.stats()
    progress("registration timed")
    host_reduce = world > 1 and os.environ.get("ICP_BENCH_HOST_REDUCE") == "1"
    its = args.steps * REGISTRATION_ITERS
    per_rank = [rank_record(rank, ctx.comm_info(), nn_avg_ms, ar_ms, c, st["iterations"], dt_local * 1e3 / its, reg)]
    if dist is not None:
        got = [None] * world
        dist.all_gather_object(got, per_rank[0])
        per_rank = got
    device_error = check_devices(per_rank, world, rccl=(world > 1 and not host_reduce) or args.rccl)
    pairs = c * args.n
    # algorithmic flop against the peak of the unit the kernel runs on
    flops = FLOP_PER_PAIR * pairs
    peak = PEAK_F16_MFMA_TFLOPS if level1 in ("mfma16", "bundle") else PEAK_FP32_TFLOPS
    achieved = flops / (nn_avg_ms * 1e-3) / 1e12 if nn_avg_ms > 0 else 0.0
    # timed iterations are seeded (the first icp_run iteration after set_scene is warm-up)
    k16 = {"plain": "nn_mfma16_kernel<seeded>", "pipe": "nn_mfma16p_kernel<seeded>",
           "unroll": "nn_mfma16x_kernel<seeded>", "r4": "nn_mfma16r_kernel<4>"}.get(
        os.environ.get("ICP_MFMA16_KERNEL", ""), "nn_mfma16r_kernel<8>")
    kernel = {"mfma16": k16, "mfma": "nn_mfma_kernel",
              "bundle": "nn_bundle_kernel" if bundle_v1() else "nn_bundle2_kernel"}.get(
        level1, "nn_fp64_kernel" if args.nn == "fp64" else "nn_filter_kernel")
    if level1 == "grid":
        # timed iterations are seeded (warm-up leaves every query a correspondence): the seeded
        # resolve (launch_nn_grid_resolve_all) scans each query's complete candidate box; AUTO
        # takes it by icp_run's policy once the scene is near the model
        kernel = grid_kernel()
    # the capture of this workload's kernels: C4 on one GPU, or rank 0's shard of the 8-way C5
    traffic_cfg = {(1 << 20, 1): "", (1 << 23, 8): "c5shard"}.get((args.n, world))
    traffic, traffic_src = pmc_traffic(kernel, traffic_cfg) if traffic_cfg is not None else (None, None)
    nn_s = nn_avg_ms * 1e-3
    compulsory = 16.0 * c + 12.0 * args.n  # §8d: fp32 xyz in (scene shard + model), int32 index out
    nn_hbm = {"compulsory_bytes": compulsory,
              "compulsory_gbps": compulsory / nn_s / 1e9 if nn_s > 0 else None,
              "pmc_bytes": traffic,
              "pmc_gbps": traffic / nn_s / 1e9 if traffic and nn_s > 0 else None,
              "peak_gbps": 8000.0,
              "pmc_hbm_frac": traffic / nn_s / 1e9 / 8000.0 if traffic and nn_s > 0 else None,
              "note": ("the bundle filter is latency-bound (dependent L2/MALL operand loads -> MFMA -> ballot per "
                       "fired block, DESIGN §3.1.1): neither HBM nor the matrix pipe is its limit"
                       if level1 == "bundle" else
                       "the O(N*M) filter is compute-bound: its HBM fraction is small by construction (§8d)")}
    dtype = {"mfma16": "f16 hi/lo-split MFMA filter (fp32 accumulate); fp64 certificate, resolve and reductions",
             "bundle": "f16 hi/lo-split MFMA bundle bound + pair filter (fp32 accumulate); fp64 certificate, "
                       "resolve and reductions",
             "mfma": "f32 MFMA filter; fp64 certificate, resolve and reductions"}.get(
        level1, "f64" if args.nn == "fp64" else "f32 VALU filter; fp64 certificate, resolve and reductions")

    workload = {1 << 20: "C4", 1 << 23: "C5"}.get(args.n, "custom")
    if rank == 0:
        out = {
            "metric": f"ICP iterations/sec (synthetic {args.n}-point pair{', ' + workload if workload != 'custom' else ''}, "
                      "exact NN)",
            "value": its / dt,
            "unit": "ICP iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "step": f"one complete registration of {REGISTRATION_ITERS} ICP iterations from device-resident clouds: "
                    "icp_set_model_device (every model image) + icp_set_scene_device + icp_run(30); "
                    "value = steps x 30 iterations / the max-over-ranks wall time; the clock EXCLUDES the PCIe "
                    "copy of the clouds (value_pcie_inclusive: the same registration from host arrays)",
            "iterations_per_step": REGISTRATION_ITERS,
            "ms_per_iteration": dt * 1e3 / its,
            "steady_state": {"iterations_per_s": STEADY_ITERS / dt_ss, "ms_per_iteration": dt_ss * 1e3 / STEADY_ITERS,
                             "iterations": STEADY_ITERS,
                             "definition": "seeded iterations of the last registration continued (no set_model / "
                                           "set_scene / unseeded first search): round 4's headline"},
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (mt19937_64 seed 42, uniform [-1,1]^3; scene = 5deg rotation + translation)",
            "config": {"workload": f"{workload} synthetic "
                                   f"{args.n}-pt model vs rigid-transformed copy, fixed iterations",
                       "n_model": args.n, "n_scene": args.n, "nn_mode": args.nn, "nn_variant": args.variant,
                       "parallelism": f"scene-sharded x{world}, model replicated, "
                                      + ("gloo host all-reduce (rehearsal)" if os.environ.get("ICP_BENCH_HOST_REDUCE") == "1" and world > 1
                                         else "RCCL all-reduce" if world > 1 or args.rccl else "no all-reduce (1 rank)")
                                      + " of 18 fp64 sums/iter"},
            "roofline": {"bound": "mfma" if level1 in ("mfma16", "mfma") else "valu",
                         "compute_unit": {"mfma16": "v_mfma_f32_32x32x16_f16 (hi/lo split, 14 products/pair) + joint v_min3 skip test (1 VALU per 2 pair values)",
                                          "mfma": "v_mfma_f32_16x16x4_f32 (G = |m|^2 - 2p.m, 4 fma/pair)"}.get(
                             level1, "VALU fp64" if args.nn == "fp64" else "VALU fp32 direct form (peak = f32 MFMA peak)"),
                         "kernel": kernel,
                         "achieved": achieved,
                         "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": traffic,
                         "traffic_unit": "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE)", "traffic_source": traffic_src,
                         "avg_launch_ms": nn_avg_ms, "flop_per_launch": flops,
                         "flop_definition": "algorithmic: 8 flop per (query, model) pair (SURVEY.md §8d); "
                                            f"pairs = {c} local queries x {args.n} model points",
                         "pairs_per_s": pairs / nn_s if nn_s > 0 else 0.0,
                         "nn_hbm": nn_hbm},
            "per_rank": per_rank,
            "mfma_uncertified_per_iter": st["level1_queued"] / max(st["iterations"], 1),
            "fp64_resolved_per_iter": st["ambiguous"] / max(st["iterations"], 1),
            "final_err": float(errs[-1]) if errs.size else None,
        }
        out["step_phases"] = dict(reg_dev)
        out["step_paths"] = {"run_grid_searches": path_st["run_grid_searches"],
                             "run_bundle_searches": path_st["run_bundle_searches"],
                             "run_certified": path_st["run_certified"], "run_walked": path_st["run_walked"],
                             "run_path_bits": hex(path_st["run_path_bits"]),
                             "note": "one registration after the timed region (icp_stats)"}
        out["step_phases"]["note"] = ("the headline step's phases from device-resident clouds (median of 3 "
                                      "registrations after the timed region): set_model_device, set_scene_device, "
                                      "first (unseeded) iteration, seeded iterations")
        if reg is not None:  # (host arrays in: the PCIe copy of both clouds included)
            regs = [r for r in per_rank if r.get("registration_ms")]
            out["registration"] = dict(reg)
            out["registration"]["note"] = ("PCIe-inclusive: icp_set_model / icp_set_scene from host arrays; the "
                                           "headline's steps take the same clouds from HBM")
            if world > 1:  # the job's registration: its slowest rank
                worst = max(regs, key=lambda r: r["registration_ms"])
                out["registration"].update({"rank0": reg["registration_ms"], "max_rank": worst["rank"],
                                            "registration_ms": worst["registration_ms"],
                                            "set_model_ms_max": max(r["set_model_ms"] for r in regs)})
                out["registration"]["iterations_per_s_inclusive"] = reg["iterations"] / (worst["registration_ms"] * 1e-3)
            out["value_pcie_inclusive"] = out["registration"]["iterations_per_s_inclusive"]
        if level1 == "bundle" and nn_s > 0:
            out["roofline"].update(bundle_roofline(c, args.n, nn_s, work, v1=bundle_v1()))
        if level1 == "mfma16" and nn_s > 0:
            ex = MFMA16_FLOP_PER_PAIR * pairs / nn_s / 1e12
            out["roofline"]["mfma_pipe"] = {
                "executed_tflops": ex, "util": ex / PEAK_F16_MFMA_TFLOPS,
                "note": "v_mfma_f32_32x32x16_f16 executes 32 flop per pair (K = 16, 14 slots used): "
                        "matrix-pipe utilisation, not the roofline fraction"}
        if args.nn == "certified" and args.variant == "auto" and world == 1 and args.n == 1 << 20:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            try:
                import roofline as RF
                rf = RF.roofline(None, args.n, world)
            except Exception as e:  # a missing / malformed profile must not break the bench line
                rf = {"error": str(e)}
            if rf and "kernels" in rf:
                keep = ("shifted_moments_kernel", "gather_moments_kernel", "centred_moments_kernel",
                        "transform_err_kernel", "canon_moments_kernel", "canon_transform_kernel",
                        "gather_aos_kernel")
                out["streaming"] = {"source": f"profiles/{rf['tag']}_bench_kernel_stats.csv + "
                                              f"profiles/{rf['tag']}_pmc_traffic.json (tools/roofline.py)",
                                    "kernels": {k: v for k, v in rf["kernels"].items() if k in keep}}
        if level1 == "grid":
            out["roofline"] = grid_roofline(c, args.n, nn_avg_ms, traffic, traffic_src, args.variant == "grid")
            out["dtype"] = "f64 (" + path_description(path_st) + ")"
        if world == 1 and not args.no_cow:
            out["cow_frame_rate"] = cow_frame_rate(local)
        if world == 1 and not args.no_cases:
            out["reference_cases"] = reference_cases_gpu()
            out["baseline_configs"] = baseline_configs(local)
            out["csv_io"] = csv_io(m)
            if args.variant != "grid" and args.nn == "certified":
                out["grid_nn"] = grid_nn_rate(local, m, p, args.steps)
            if level1 == "bundle":
                out["full_nxm_filter"] = full_nxm_rate(local, m, p)
        if not args.no_cpu_baseline:  # rank 0 at every N: the same host-side baseline
            out["cpu_baseline"] = cpu_baseline(m, p)
            if not args.no_cases:
                out["cpu_baseline"]["reference_cases_cpu"] = reference_cases_cpu()
            out["gpu_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            if "all_cores" in out["cpu_baseline"]:
                out["gpu_vs_cpu_all_cores"] = out["value"] / out["cpu_baseline"]["all_cores"]["value"]
        if device_error:
            out["device_error"] = device_error
        print(json.dumps(out), flush=True)
    if dist is not None:
        # rank 0 spent its CPU-baseline time above: every rank reaches the RCCL communicator's
        # destroy together rather than some destroying while a peer is still inside the job
        dist.barrier()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    if device_error:
        # the line was printed (with device_error) for the record, but the run did not measure
        # what it claims: N ranks of RCCL on N distinct GPUs
        print(f"[bench] {device_error}", file=sys.stderr)
        sys.exit(3)


def reap_children():
    """Leave no process behind (the driver counts processes at the end of the run): every child
    is joined where it is started (subprocess.run, with-block thread pools); anything still
    alive here is named on stderr and terminated."""
    try:
        import psutil
    except ImportError:
        return
    kids = psutil.Process().children(recursive=True)
    for k in kids:
        try:
            print(f"[bench] terminating leftover child {k.pid} {k.name()}", file=sys.stderr)
            k.terminate()
        except psutil.NoSuchProcess:
            pass
    psutil.wait_procs(kids, timeout=5)


if __name__ == "__main__":
    try:
        main()
    finally:
        reap_children()
