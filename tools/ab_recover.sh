#!/usr/bin/env bash
# Same-box A/B of the f16 filter's index recovery (batched, out of line) against a baseline
# library (tools/build_ab.sh REV): GPU tests, C4 bench, W = 1 / 8 shard probe.
#   usage: tools/ab_recover.sh TAG BASELINE_LIB
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab_recover}; BASE=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    case $rc in 0) ;; 1) [ "$name" = pytest ] || exit 1 ;; *) tail -n 20 "$OUT/$name.log"; exit $rc ;; esac
    tail -n 3 "$OUT/$name.log" | cut -c1-300
}
step pytest 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread
B="python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cow --no-cases"
for r in 1 2; do
    ICP_AMD_LIB=$BASE step bench_base_$r 300 $B
    step bench_new_$r 300 $B
done
for r in 1 2; do
    ICP_AMD_LIB=$BASE step shard_base_$r 300 python3 tools/shard_probe.py --worlds 8 4 --steps 20
    step shard_new_$r 300 python3 tools/shard_probe.py --worlds 8 4 --steps 20
done
