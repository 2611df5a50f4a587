#!/usr/bin/env bash
# The round's measurement capture of the default C4 bench (one GPU), each GPU step under its own
# time limit, written under gpurun_out/TAG and profiles/:
#   1. rocprofv3 kernel trace + stats of bench.py      -> profiles/TAG_bench_kernel_stats.csv
#   2. FETCH_SIZE and WRITE_SIZE passes (separately)   -> profiles/TAG_pmc_traffic.json (pmc_summary.py)
#   3. SQ / TA / TD / TCP / TCC passes of the fused kernel (pmc_probe.sh) -> profiles/TAG_sq_iter.json
#   4. the default bench line (it reads 1-2's files)   -> profiles/TAG/bench.log
#   usage: tools/capture_round.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p "$O" "profiles/$TAG"; export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases"
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    case $rc in 0) ;; 124|137|134|139) echo "fatal: stopping"; exit $rc ;; esac
}
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench -- $B
cp "$(find "$O/trace" -name 'bench_kernel_stats.csv' | head -1)" "profiles/${TAG}_bench_kernel_stats.csv"
step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o f -- $B --no-registration
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o w -- $B --no-registration
python3 tools/pmc_summary.py "$(find "$O/fetch" -name '*counter_collection.csv' | head -1)" \
    "$(find "$O/write" -name '*counter_collection.csv' | head -1)" "profiles/${TAG}_pmc_traffic.json"
step sq 600 bash tools/pmc_probe.sh "$TAG/sq" nn_grid_iter2
python3 tools/sq_summary.py "profiles/${TAG}_sq_iter.json" "$O"/sq/p*/p_counter_collection.csv > /dev/null
step bench 400 python3 bench.py
cp "$O/bench.log" "profiles/$TAG/bench.log"
echo done
