set -u
O=gpurun_out/ab_strands2; mkdir -p $O
for k in 1 2; do
 for cfg in "s16k ICP_ITER_XCD_L=16" "s16k ICP_ITER_XCD_L=32" "s16k ICP_ITER_XCD_L=64" "s32k -" "s32k ICP_ITER_XCD_L=32" "s32k ICP_ITER_XCD_L=128"; do
  set -- $cfg; v=$1; e=$2; a=""; [ "$e" != - ] && a=$e
  tag=${v}_$(echo $e | tr '=' '_')
  env $a ICP_AMD_LIB=iterative-closest-point_amd/build_ab/$v/libicp_hip.so timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cow --no-cases > $O/bench_${tag}_$k.log 2>&1 || exit 1
  env $a ICP_AMD_LIB=iterative-closest-point_amd/build_ab/$v/libicp_hip.so timeout -k 10 200 python -u tools/shard_probe.py --worlds 1 8 > $O/shard_${tag}_$k.log 2>&1 || exit 1
 done
done
echo done
