set -u
# Seeded grid variant: lanes per query (ICP_GRID_GROUP) x scan form (ICP_GRID_SCAN) at C4, C2, C3.
O=gpurun_out/${1:-r01eg}; mkdir -p $O
for g in 4 1 16; do for sc in rows flat; do
  ICP_GRID_GROUP=$g ICP_GRID_SCAN=$sc timeout -k 10 200 python bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/g${g}_$sc.log 2>&1 || exit 1
  ICP_GRID_GROUP=$g ICP_GRID_SCAN=$sc timeout -k 10 300 python tools/configs_probe.py --configs C2_bunny C3_horse --variants grid --reps 3 >> $O/g${g}_$sc.log 2>&1 || exit 1
done; done
echo done
