#!/usr/bin/env python3
"""Per-kernel SQ counters from rocprofv3 --pmc passes, averaged over launches, with the derived
issue figures DESIGN.md quotes (instructions per MFMA, wait share, effective clock).

    python tools/sq_summary.py OUT.json PASS1_counter_collection.csv [PASS2 ...] [--kernel NAME]

GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md): cycles per launch = /8.
"""
import collections
import csv
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_summary import short  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else None
    if kernel:
        args.remove(kernel)
    out_path, paths = args[0], args[1:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        if kernel and k != kernel:
            continue
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["launches"] = max(len(v) for v in cs.values())
        mf = d.get("SQ_INSTS_MFMA")
        if mf:
            d["valu_per_mfma"] = d.get("SQ_INSTS_VALU", 0.0) / mf
            d["salu_per_mfma"] = d.get("SQ_INSTS_SALU", 0.0) / mf
        if d.get("SQ_WAVE_CYCLES"):
            d["wait_share"] = d.get("SQ_WAIT_ANY", 0.0) / d["SQ_WAVE_CYCLES"]
        if d.get("GRBM_GUI_ACTIVE"):
            d["gpu_cycles_per_launch"] = d["GRBM_GUI_ACTIVE"] / 8.0
        res[k] = d
    json.dump({"source": paths, "kernels": res}, open(out_path, "w"), indent=1, sort_keys=True)
    for k, d in res.items():
        print(k, {x: round(d[x], 3) for x in ("valu_per_mfma", "salu_per_mfma", "wait_share") if x in d})


if __name__ == "__main__":
    main()
