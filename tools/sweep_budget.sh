# Grid box budget sweep (ICP_GRID_BUDGET, cells) at C2 / C3, auto and grid variants.
set -u
O=gpurun_out/${1:-r01dr}; mkdir -p $O
for b in 6060 12000 24000 65536 200000; do
  ICP_GRID_BUDGET=$b timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse --variants auto grid --reps 3 > $O/b$b.log 2>&1 || exit 1
done
echo done
