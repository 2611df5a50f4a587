# A/B of the seeded grid kernel's forms (ICP_GRID_SEEDED = "G,KR,KU[,waves]") and of the XCD
# block remap (ICP_GRID_XCD = 0 | 1 | 2) on the C4 bench iteration and the 8-way shard probe.
#   tools/seeded_ab.sh TAG "form1 form2 ..."
set -u
O=gpurun_out/${1:-ab}; mkdir -p $O; export TMPDIR=/tmp
FORMS=${FORMS:-${2:-"2,2,2 f2,2,2 4,2,2 f4,2,2 4,1,2 f4,1,2"}}
# the whole GPU suite on the defaults, then the exactness of the other forms (the policy
# tests compare bit for bit)
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { echo "GPU tests failed"; tail -15 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for f in $FORMS; do
  ICP_GRID_SEEDED=$f timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_grid_policy.py > $O/t_$f.log 2>&1 || { echo "form $f: tests failed"; tail -5 $O/t_$f.log; exit 1; }
done
line() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['per_rank'][0]
        print(f\"{sys.argv[2]:>14s} it/s {d['value']:8.1f} ms/step {d['ms_per_step']*1e3:7.1f}us grid {r['filter_ms']*1e3:7.1f}us tail {r['tail_ms']*1e3:6.1f}us\")
" $1 "$2"; }
shard8() { python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l)
        if d['world'] == 8:
            print(f\"{sys.argv[2]:>14s} W=8 ms/iter {d['ms_per_iter']*1e3:7.1f}us grid {d['filter_ms']*1e3:7.1f}us other {d['other_ms']*1e3:6.1f}us\")
" $1 "$2"; }
for f in $FORMS; do
  ICP_GRID_SEEDED=$f timeout -k 10 120 python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-cow --no-cases --no-registration > $O/b_$f.log 2>&1 || exit 1
  line $O/b_$f.log "$f" | tee -a $O/summary.txt
  ICP_GRID_SEEDED=$f timeout -k 10 120 python3 tools/shard_probe.py --worlds 8 --steps 30 > $O/s_$f.log 2>&1 || exit 1
  shard8 $O/s_$f.log "$f" | tee -a $O/summary.txt
done
for fs in ${FUSED:-1 2 3}; do
  ICP_FUSED_STEPS=$fs timeout -k 10 120 python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-cow --no-cases --no-registration > $O/b_fused$fs.log 2>&1 || exit 1
  line $O/b_fused$fs.log "fused=$fs" | tee -a $O/summary.txt
  ICP_FUSED_STEPS=$fs timeout -k 10 120 python3 tools/shard_probe.py --worlds 8 --steps 30 > $O/s_fused$fs.log 2>&1 || exit 1
  shard8 $O/s_fused$fs.log "fused=$fs" | tee -a $O/summary.txt
done
for x in 0 2; do
  ICP_GRID_XCD=$x timeout -k 10 120 python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-cow --no-cases --no-registration > $O/b_xcd$x.log 2>&1 || exit 1
  line $O/b_xcd$x.log "xcd=$x" | tee -a $O/summary.txt
done
timeout -k 10 200 python3 tools/shard_probe.py --worlds 1 8 --steps 30 > $O/shard.log 2>&1 || exit 1
echo done
