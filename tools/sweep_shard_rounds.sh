# 8-way C4 shard (rank 0's 131,072 queries vs the full model): split-plan rounds sweep.
set -u
O=gpurun_out/${1:-r01dt}; mkdir -p $O
for r in 4 2 3 6 8 4; do
  ICP_NN_MIN_ROUNDS=$r timeout -k 10 300 python tools/shard_probe.py --worlds 8 4 --steps 20 >> $O/rounds_$r.log 2>&1 || exit 1
done
echo done
