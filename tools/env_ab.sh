# A/B of one environment switch on the C4 bench iteration (60 steps) and the W = 8 shard:
#   tools/env_ab.sh TAG VAR "v1 v2 ..."
set -u
O=gpurun_out/${1:-envab}; VAR=$2; VALS=$3; mkdir -p $O; export TMPDIR=/tmp
for v in $VALS; do
  env $VAR=$v timeout -k 10 120 python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-cow --no-cases --no-registration > $O/b_$v.log 2>&1 || exit 1
  env $VAR=$v timeout -k 10 120 python3 tools/shard_probe.py --worlds 8 --steps 30 --warmup 5 > $O/s_$v.log 2>&1 || exit 1
  python3 - "$O/b_$v.log" "$O/s_$v.log" "$VAR=$v" <<'PY' | tee -a $O/summary.txt
import json, sys
b = s = None
for l in open(sys.argv[1]):
    if l.startswith('{'): b = json.loads(l)
for l in open(sys.argv[2]):
    if l.startswith('{'): s = json.loads(l)
r = b['per_rank'][0]
print(f"{sys.argv[3]:>22s} W=1 {b['ms_per_step']*1e3:6.1f}us (grid {r['filter_ms']*1e3:6.1f} tail {r['tail_ms']*1e3:5.1f})  "
      f"W=8 {s['ms_per_iter']*1e3:6.1f}us (grid {s['filter_ms']*1e3:5.1f} other {s['other_ms']*1e3:5.1f})")
PY
done
echo done
