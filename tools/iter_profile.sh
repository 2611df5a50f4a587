# Per-iteration cost of the C4 path and its W-way shards on one GPU: shard_probe (auto and
# grid variants, 1-rank RCCL) and rocprofv3 kernel traces of rank 0's W = 8 shard and of the
# bench's C4 iterations (tools/timeline.py reads them).   tools/iter_profile.sh TAG
set -u
O=gpurun_out/${1:-r04x}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python3 tools/shard_probe.py --worlds 1 2 4 8 --steps 30 > $O/shard_auto.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/shard_probe.py --worlds 1 2 4 8 --steps 30 --variant grid > $O/shard_grid.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o shard8 -- python3 tools/shard_probe.py --worlds 8 --steps 20 > $O/prof_shard8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cow --no-cases --no-registration > $O/prof_c4.log 2>&1 || exit 1
echo done
