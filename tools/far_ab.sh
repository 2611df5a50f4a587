# The search policy's far threshold (ICP_GRID_FAR_SHIFT: n >> shift) on the default bench
# (30 steps after 3 warm-up) with its registration block, and the W = 8 shard.
set -u
O=gpurun_out/${1:-farab}; mkdir -p $O; export TMPDIR=/tmp
VALS=${2:-"5 3 2 1 0"}
for v in $VALS; do
  ICP_GRID_FAR_SHIFT=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-cow --no-cases > $O/b_$v.log 2>&1 || exit 1
  python3 - "$O/b_$v.log" "shift=$v" <<'PY' | tee -a $O/summary.txt
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'): b = json.loads(l)
r = b['registration']
print(f"{sys.argv[2]:>9s} bench {b['value']:7.1f} it/s ({b['ms_per_step']*1e3:6.1f} us)  registration {r['iterations_per_s_inclusive']:7.1f} it/s "
      f"(first {r['first_iteration_ms']:.3f} ms, seeded {r['seeded_iteration_ms']*1e3:6.1f} us)")
PY
done
echo done
