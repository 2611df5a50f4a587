# C3 (horse_ref vs horse_tr1, 50 iterations): rocprofv3 kernel trace + the two PMC passes for
# per-kernel HBM bytes (BASELINE config C3's "rocprof HBM-GB/s capture"), and the one-launch
# kernel's phase stamps; the summaries are written where tools/roofline.py --config C3 and
# bench.py's baseline_configs read them: profiles/TAG_c3_{kernel_stats.csv,pmc_traffic.json,stamps.stamps}.
#   usage: tools/c3_hbm.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
P="python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c3 -- $P > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc1 -o fetch -- $P > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc2 -o write -- $P > $O/pmc2.log 2>&1 || exit 1
ICP_PERSIST_STAMPS=1 timeout -k 10 120 $P > $O/stamps.log 2>&1 || exit 1
cp "$(find $O/trace -name 'c3_kernel_stats.csv' | head -1)" "profiles/${TAG}_c3_kernel_stats.csv"
python3 tools/pmc_summary.py "$(find $O/pmc1 -name '*counter_collection.csv' | head -1)" \
    "$(find $O/pmc2 -name '*counter_collection.csv' | head -1)" "profiles/${TAG}_c3_pmc_traffic.json" > /dev/null || exit 1
grep '^\[persist' $O/stamps.log > "profiles/${TAG}_c3_stamps.stamps"
cp $O/trace.log "profiles/${TAG}_c3_probe.log"
echo done
