# Same-box A/B of environment settings: the C4 bench line and the W = 1 / 8 shard probe for each,
# alternating, twice.   tools/ab_envs.sh TAG 'VAR=a' 'VAR=b' ...   ('-' = no setting; '+' joins several)
set -u
O=gpurun_out/$1; shift; mkdir -p $O
for k in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e" | tr '=,+' '___'); env_args=""; [ "$e" != - ] && env_args=$(echo "$e" | tr '+' ' ')
    env $env_args timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cow --no-cases > $O/bench_${tag}_$k.log 2>&1 || exit 1
    env $env_args timeout -k 10 200 python -u tools/shard_probe.py --worlds 1 8 > $O/shard_${tag}_$k.log 2>&1 || exit 1
  done
done
echo done
