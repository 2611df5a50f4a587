set -u
O=gpurun_out/r01cz; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTFAIL; tail -30 $O/pytest.log; exit 1; }
for mode in flat rows flat rows; do
  ICP_GRID_SCAN=$mode timeout -k 10 200 python tools/configs_probe.py --configs C2_bunny C3_horse --variants auto grid >> $O/configs_$mode.log 2>&1 || exit 1
  ICP_GRID_SCAN=$mode timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases >> $O/bench_$mode.log 2>&1 || exit 1
done
echo done
