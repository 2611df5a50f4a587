#!/usr/bin/env bash
# C5 (8M-point pair) as an 8-rank job on ONE GPU: torchrun, scene sharded 8 ways, the per-iteration
# sums through gloo (ICP_BENCH_HOST_REDUCE=1) since RCCL needs one GPU per rank.  The ranks share
# the card, so ms_per_step is ~8x a real 8-GPU step; per_rank filter times are each shard's own.
#   usage: tools/c5_rehearsal.sh TAG [ranks]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02c5}
RANKS=${2:-8}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# the job prints once, at its end: a progress line a minute keeps the call visibly alive
(for i in $(seq 1 14); do sleep 45; echo "[c5_rehearsal] $((45 * i)) s"; done) &
TICK=$!
ICP_BENCH_HOST_REDUCE=1 timeout -k 10 660 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$RANKS" \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$RANKS" --points 8388608 --steps 5 --warmup 1 \
    > "$OUT/bench_c5_dist$RANKS.log" 2>&1
rc=$?
kill $TICK 2>/dev/null
wait $TICK 2>/dev/null
echo "bench rc=$rc"
tail -c 3000 "$OUT/bench_c5_dist$RANKS.log"
exit $rc
