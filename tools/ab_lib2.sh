# Same-box A/B of the working tree's library against build_ab/REV: GPU tests (new lib), then
# C2/C3 auto + grid variant and the C4 grid variant for both libraries.
#   tools/ab_lib2.sh TAG REV
set -u
O=gpurun_out/$1; REV=$2; mkdir -p $O
OLD=iterative-closest-point_amd/build_ab/$REV/libicp_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for k in 1 2; do
  timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse --variants auto grid --reps 3 >> $O/new.log 2>&1 || exit 1
  ICP_AMD_LIB=$OLD timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse --variants auto grid --reps 3 >> $O/old.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/grid_new.log 2>&1 || exit 1
ICP_AMD_LIB=$OLD timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/grid_old.log 2>&1 || exit 1
echo done
