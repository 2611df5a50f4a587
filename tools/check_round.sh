# Full GPU test suite, then the mid-size configs and the C4 grid variant.
set -u
O=gpurun_out/${1:-r01dj}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse --variants auto grid --reps 3 > $O/configs.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/bench_grid.log 2>&1 || exit 1
echo done
