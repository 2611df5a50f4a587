#!/usr/bin/env python3
"""icp_set_model's device timeline from a rocprofv3 kernel + memory-copy trace of
tools/registration_probe.py: every kernel and copy from the K-th model_stats_kernel dispatch
(the start of a set_model) up to the next make_f32 / query_keys (the scene's upload).

    python tools/setmodel_timeline.py PROF_DIR/PREFIX [--nth K]
"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="e.g. gpurun_out/r04d/prof/reg (…_kernel_trace.csv, …_memory_copy_trace.csv)")
    ap.add_argument("--nth", type=int, default=1)
    ap.add_argument("--anchor", default="model_stats_kernel")
    ap.add_argument("--end", default="aos_to_soa_f32_kernel|make_f32_kernel")
    a = ap.parse_args()
    ev = []
    for path in glob.glob(a.prefix + "*kernel_trace.csv"):
        for x in csv.DictReader(open(path)):
            ev.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"]))
    for path in glob.glob(a.prefix + "*memory_copy_trace.csv"):
        for x in csv.DictReader(open(path)):
            nb = x.get("Bytes") or x.get("Size") or ""
            ev.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]),
                       f"COPY {x.get('Direction', '')} {nb} B"))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if a.anchor in e[2]]
    i0 = starts[a.nth]
    ends = a.end.split("|")
    i1 = next(i for i in range(i0 + 1, len(ev)) if any(s in ev[i][2] for s in ends))
    # the copy that fed this set_model: the last host-to-device copy before the anchor
    j = max(i for i in range(i0) if ev[i][2].startswith("COPY"))
    t0 = ev[j][0]
    busy = 0
    prev = None
    for s, e, name in ev[j:i1 + 1]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(e - s) / 1e3:8.1f}  {name[:90]}")
        busy += e - s
        prev = e
    print(f"span {(ev[i1][0] - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
