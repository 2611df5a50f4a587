# Multi-GPU evidence on one box: the C4 shard probe at W = 1/2/4/8 and C5's W = 8
# shard, registrations (host arrays) of C4 and of C5's rank-0 shard, and the 8-rank C5 flow
# rehearsed on one GPU (gloo sums).   tools/evidence_mgpu.sh TAG
set -u
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u tools/shard_probe.py --worlds 1 2 4 8 > $O/shard_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_probe.py --n 8388608 --worlds 8 --steps 5 --warmup 2 > $O/shard_c5.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/registration_probe.py > $O/reg_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/registration_probe.py --points 8388608 --world 8 --reps 4 > $O/reg_c5_shard.log 2>&1 || exit 1
ICP_BENCH_HOST_REDUCE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --points 8388608 --steps 10 --warmup 2 \
    --no-cpu-baseline --no-cow --no-cases > $O/bench_c5_dist8.log 2>&1 || exit 1
echo done
