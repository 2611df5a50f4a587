# The seeded grid kernel's forms at rank 0's shard of the 8-way C5 (2^20 queries, 2^23 model):
#   tools/c5_forms.sh TAG "form1 form2 ..."
set -u
O=gpurun_out/${1:-c5f}; mkdir -p $O; export TMPDIR=/tmp
FORMS=${2:-"2,2,2 f2,2,2 f4,2,2 4,2,2"}
for f in $FORMS; do
  ICP_GRID_SEEDED=$f timeout -k 10 200 python3 tools/shard_probe.py --n 8388608 --worlds 8 --steps 12 --warmup 8 > $O/c5_$f.log 2>&1 || exit 1
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(f\"{sys.argv[2]:>8s} C5 shard ms/iter {d['ms_per_iter']*1e3:7.1f}us grid {d['filter_ms']*1e3:7.1f}us other {d['other_ms']*1e3:6.1f}us last {d['last_filter']}\")
" $O/c5_$f.log "$f" | tee -a $O/summary.txt
done
echo done
