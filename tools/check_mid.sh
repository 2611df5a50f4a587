set -u
O=gpurun_out/r01dd; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
CFG="C2_bunny C3_horse syn16384 syn65536" timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse syn16384 syn65536 --variants auto --reps 3 > $O/configs.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_horse -o horse -- \
    python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 3 > $O/prof_horse.log 2>&1 || exit 1
echo done
