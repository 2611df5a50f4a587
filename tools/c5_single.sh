# C5 scale check on ONE GPU: the full 8M x 8M search (world 1) and rank 0's 8-way shard.
set -u
O=gpurun_out/${1:-r01dx}; mkdir -p $O
timeout -k 10 600 python3 tools/shard_probe.py --n 8388608 --worlds 1 8 --steps 3 --warmup 1 > $O/c5.log 2>&1 || exit 1
echo done
