"""Per-iteration kernel durations of C4 registrations (run under rocprofv3 --kernel-trace):
3 registrations of the bench's workload (synthetic 2^20 pair, 30 iterations each).  Parse the
trace with tools/iter_trace.py --parse DB_OR_CSV: the fused kernel's durations by iteration."""
import argparse
import os
import sqlite3
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "iterative-closest-point_amd"))


def run(n, regs, iters):
    import icp_amd
    m, p = icp_amd.synthetic_pair(n, seed=42, angle_deg=5.0)
    with icp_amd.Context(0) as ctx:
        for _ in range(regs):
            ctx.set_model(m)
            ctx.set_scene(p)
            ctx.run(iters, -1.0)
    print("trace ok")


def parse(path, kernel="nn_grid_iter_kernel"):
    c = sqlite3.connect(path)
    rows = list(c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                          "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    names = [r[0] for r in rows]
    # registration boundaries: the grid build's key kernel opens each
    marks = [i for i, nm in enumerate(names) if "grid_keys_kernel" in nm]
    out = []
    for a, b in zip(marks, marks[1:] + [len(rows)]):
        out.append([(rows[i][2] - rows[i][1]) / 1e3 for i in range(a, b) if kernel in names[i]])
    for k, d in enumerate(out):
        print(f"registration {k}: {len(d)} launches, us: " + " ".join(f"{x:.0f}" for x in d))
    if out:
        m = np.array([d for d in out if len(d) == len(out[-1])])
        print("mean by iteration (us):", " ".join(f"{x:.0f}" for x in m.mean(0)))
        print(f"total {m.sum(1).mean():.0f} us, first 5 {m[:, :5].sum(1).mean():.0f}, last 5 mean {m[:, -5:].mean():.1f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--regs", type=int, default=3)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--parse", default=None)
    ap.add_argument("--kernel", default="nn_grid_iter_kernel")
    a = ap.parse_args()
    if a.parse:
        parse(a.parse, a.kernel)
    else:
        run(a.n, a.regs, a.iters)
