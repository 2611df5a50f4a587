# Lanes-per-query sweep for the grid kernels (resolve: ICP_GRID_RGROUP, search: ICP_GRID_GROUP),
# plus one rocprofv3 kernel trace of C3 for the iteration timeline.
set -u
O=gpurun_out/${1:-r01da}; mkdir -p $O
for g in 16 64 4; do
  ICP_GRID_RGROUP=$g timeout -k 10 200 python tools/configs_probe.py --configs C2_bunny C3_horse --variants auto >> $O/rgroup_$g.log 2>&1 || exit 1
  ICP_GRID_RGROUP=$g timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases >> $O/bench_rgroup_$g.log 2>&1 || exit 1
done
for g in 4 16 1; do
  ICP_GRID_GROUP=$g timeout -k 10 200 python tools/configs_probe.py --configs C2_bunny C3_horse --variants grid >> $O/sgroup_$g.log 2>&1 || exit 1
  ICP_GRID_GROUP=$g timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases >> $O/bench_sgroup_$g.log 2>&1 || exit 1
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_horse -o horse -- \
    python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 3 > $O/prof_horse.log 2>&1 || exit 1
echo done
