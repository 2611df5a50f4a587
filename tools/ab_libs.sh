# Same-box A/B of the working tree's library against build_ab variants: the C4 bench line and the
# W = 1 / 8 shard probe, alternating, twice.   tools/ab_libs.sh TAG VARIANT...
set -u
O=gpurun_out/$1; shift; mkdir -p $O
for k in 1 2; do
  for v in cur "$@"; do
    L=""; [ "$v" != cur ] && L=iterative-closest-point_amd/build_ab/$v/libicp_hip.so
    ICP_AMD_LIB=$L timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cow --no-cases > $O/bench_${v}_$k.log 2>&1 || exit 1
    ICP_AMD_LIB=$L timeout -k 10 200 python -u tools/shard_probe.py --worlds 1 8 > $O/shard_${v}_$k.log 2>&1 || exit 1
  done
done
echo done
