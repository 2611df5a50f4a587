set -u
O=gpurun_out/ab_prune; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_canon.py > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cow --no-cases > $O/new_$k.log 2>&1 || exit 1
  ICP_AMD_LIB=iterative-closest-point_amd/build_ab/noprune/libicp_hip.so timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cow --no-cases > $O/old_$k.log 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/shard_probe.py > $O/shard_new.log 2>&1 || exit 1
ICP_AMD_LIB=iterative-closest-point_amd/build_ab/noprune/libicp_hip.so timeout -k 10 200 python -u tools/shard_probe.py > $O/shard_old.log 2>&1 || exit 1
echo done
