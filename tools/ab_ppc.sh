# Grid density A/B (ICP_GRID_PPC) on one box: the C4 bench line and the shard probe per density.
#   tools/ab_ppc.sh TAG PPC...
set -u
O=gpurun_out/$1; shift; mkdir -p $O
for p in "$@"; do
  ICP_GRID_PPC=$p timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cow --no-cases > $O/bench_ppc$p.log 2>&1 || exit 1
  ICP_GRID_PPC=$p timeout -k 10 200 python -u tools/shard_probe.py --worlds 1 8 > $O/shard_ppc$p.log 2>&1 || exit 1
done
echo done
