# Full GPU suite, then the given tools/gpu_round.sh steps; a fault / timeout in the suite ends it
# (test failures do not: the measurements still run).   tools/round_check.sh TAG [steps...]
set -u
T=${1:-r04x}; shift || true
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?
tail -n 3 gpurun_out/$T/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
[ "${C5F:-0}" = 1 ] && { bash tools/c5_forms.sh $T/c5f || exit 1; }
bash tools/gpu_round.sh $T "$@"
