#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): the counters are in KiB; on gfx950 FETCH_SIZE
reports half of the bytes of wide (16 B/lane) coalesced streaming reads, so it is doubled.
Every kernel here that streams bulk data reads 16 B/lane (LDS-DMA model tiles, float4/double2
loads); narrower reads are a small share of each kernel's bytes, so the doubled figure is an
upper bound for them.  WRITE_SIZE is exact for 16 B/lane stores.  Infinity-Cache (L3) hits are
counted by these counters, so for data re-read from L3 the figure is traffic out of L2, which is
an upper bound on HBM bytes.
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def short(name):
    """Kernel name without namespace or arguments.  Tags: "<list>" for the level-2 list
    variant of nn_filter_kernel, "<seeded>" for the seeded f16 filters."""
    full = name
    n = name.replace("void ", "").replace("icp::(anonymous namespace)::", "")
    if n.startswith("_ZN3icp12_GLOBAL__N_1"):  # mangled: _ZN3icp12_GLOBAL__N_1<len><name>...
        rest = n[len("_ZN3icp12_GLOBAL__N_1"):]
        digits = "".join(c for c in rest[:3] if c.isdigit())
        n = rest[len(digits):len(digits) + int(digits)]
    base = n.split("(")[0]
    tmpl = base[base.find("<"):] if "<" in base else ""
    base = base.split("<")[0]
    if base == "nn_filter_kernel" and "true" in tmpl:
        return base + "<list>"
    if base == "nn_mfma16r_kernel":  # seeded-only, template = query groups per wave
        qg = tmpl.strip("<>") or ("8" if "ILi8E" in full else "4" if "ILi4E" in full else "?")
        return f"{base}<{qg}>"
    if base.startswith("nn_mfma16") and ("<true" in tmpl or "true>" in tmpl or "Lb1E" in full):
        return base + "<seeded>"
    if base == "canon_fold_kernel" and tmpl:  # <K0, K, mode>: the iteration's fold / the first moments' folds
        return base + tmpl.replace(" ", "")
    if base == "nn_grid_resolve_kernel" and tmpl:  # lanes per query: 4 (every query), 16 / 64 (queues)
        return f"{base}<{tmpl.strip('<>').split(',')[0].strip()}>"
    return base


def main():
    fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
    write, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in fetch:
        out[short(k)] = {
            "kernel": k[:160],
            "launches": nf[k],
            "fetch_bytes_per_launch": 2.0 * fetch[k],
            "write_bytes_per_launch": write.get(k, 0.0),
            "traffic_bytes_per_launch": 2.0 * fetch[k] + write.get(k, 0.0),
        }
    json.dump({"source": [sys.argv[1], sys.argv[2]],
               "correction": "FETCH_SIZE x2 (gfx950 16 B/lane reads), KiB -> bytes",
               "kernels": out}, open(sys.argv[3], "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"]):
        print(f"{k:40s} {v['launches']:4d}  fetch {v['fetch_bytes_per_launch'] / 1e6:10.2f} MB"
              f"  write {v['write_bytes_per_launch'] / 1e6:8.2f} MB")


if __name__ == "__main__":
    main()
