# Fused single-rank passes (last-workgroup fold) vs separate reduce / Horn / error launches.
set -u
O=gpurun_out/${1:-r01de}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for f in 1 0 1 0; do
  ICP_FUSED_PASSES=$f timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse syn16384 syn65536 --variants auto --reps 3 >> $O/configs_$f.log 2>&1 || exit 1
done
ICP_FUSED_PASSES=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/bench_1.log 2>&1 || exit 1
ICP_FUSED_PASSES=0 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/bench_0.log 2>&1 || exit 1
echo done
