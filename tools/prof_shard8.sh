set -u
O=gpurun_out/r01dv; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o shard -- python3 tools/shard_probe.py --worlds 8 --steps 20 > $O/shard.log 2>&1 || exit 1
echo done
