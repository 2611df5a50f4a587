# The seeded grid kernel's forms at C4's W-way shards (rank 0's shard, 1-rank RCCL):
#   tools/shard_forms.sh TAG "form1 form2 ..." "worlds"
set -u
O=gpurun_out/${1:-shf}; mkdir -p $O; export TMPDIR=/tmp
FORMS=${2:-"4,2,2 f4,2,2 4,1,2 f4,1,2 2,2,2"}
WORLDS=${3:-"2 4 8"}
for f in $FORMS; do
  ICP_GRID_SEEDED=$f timeout -k 10 200 python3 tools/shard_probe.py --worlds $WORLDS --steps 30 --warmup 5 > $O/sh_$f.log 2>&1 || exit 1
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(f\"{sys.argv[2]:>8s} W={d['world']} ms/iter {d['ms_per_iter']*1e3:7.1f}us grid {d['filter_ms']*1e3:7.1f}us other {d['other_ms']*1e3:6.1f}us\")
" $O/sh_$f.log "$f" | tee -a $O/summary.txt
done
echo done
