# C4: flattened vs per-row grid scans, for the grid variant (search kernel) and the unseeded
# search (grid seed kernel + seeded filter).
set -u
O=gpurun_out/${1:-r01dh}; mkdir -p $O
for mode in flat rows flat rows; do
  ICP_GRID_SCAN=$mode timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases >> $O/grid_$mode.log 2>&1 || exit 1
  ICP_GRID_SCAN=$mode timeout -k 10 200 python tools/nn_probe.py --variant mfma16 --reps 3 >> $O/probe_$mode.log 2>&1 || exit 1
done
echo done
