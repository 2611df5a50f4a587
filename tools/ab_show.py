"""Summarise tools/ab_libs.sh / ab_ppc.sh logs: tools/ab_show.py gpurun_out/TAG"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
    ls = [x for x in open(f) if x.startswith("{")]
    if not ls:
        print(os.path.basename(f), "no line"); continue
    j = json.loads(ls[-1]); ph = j.get("step_phases", {})
    sh = f.replace("bench_", "shard_")
    w = []
    if os.path.exists(sh):
        w = [(json.loads(x)["world"], round(json.loads(x)["ms_per_iter"], 4)) for x in open(sh) if x.startswith('{"world"')]
    print(f"{os.path.basename(f):28s} {j['value']:7.0f} it/s  seeded {ph.get('seeded_iteration_ms', 0):.4f}  "
          f"first {ph.get('first_iteration_ms', 0):.3f}  steady {j.get('steady_state', {}).get('ms_per_iteration', 0):.4f}  "
          f"roof {j['roofline']['achieved']:.0f}  {w}")
