# rocprofv3 kernel trace of rank 0's 8-way C4 shard (131,072 queries vs the full model) on one
# GPU, for the per-iteration timeline (tools/timeline.py).   tools/prof_shard8.sh [TAG]
set -u
O=gpurun_out/${1:-r01dv}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o shard -- python3 tools/shard_probe.py --worlds 8 --steps 20 > $O/shard.log 2>&1 || exit 1
echo done
