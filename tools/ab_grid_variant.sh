set -u
# Grid-variant A/B (seeded vs the build_ab/HEAD library) after the full GPU suite.
O=gpurun_out/${1:-r01ef}; mkdir -p $O
OLD=iterative-closest-point_amd/build_ab/HEAD/libicp_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for k in 1 2; do
  timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse C1_cow_gpu --variants grid --reps 3 >> $O/new.log 2>&1 || exit 1
  ICP_AMD_LIB=$OLD timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse C1_cow_gpu --variants grid --reps 3 >> $O/old.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases >> $O/grid_new.log 2>&1 || exit 1
  ICP_AMD_LIB=$OLD timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases >> $O/grid_old.log 2>&1 || exit 1
done
echo done
