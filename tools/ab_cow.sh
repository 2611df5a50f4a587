# Cow-size A/B of the working tree's library against build_ab/REV (after the parity/sharded GPU
# tests): complete registrations (C1 cow, 2x4096 synthetic).   tools/ab_cow.sh TAG REV
set -u
O=gpurun_out/$1; REV=$2; mkdir -p $O
OLD=iterative-closest-point_amd/build_ab/$REV/libicp_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for k in 1 2 3; do
  timeout -k 10 300 python tools/configs_probe.py --configs C1_cow_gpu syn4096 --variants auto --reps 20 >> $O/new.log 2>&1 || exit 1
  ICP_AMD_LIB=$OLD timeout -k 10 300 python tools/configs_probe.py --configs C1_cow_gpu syn4096 --variants auto --reps 20 >> $O/old.log 2>&1 || exit 1
done
echo done
