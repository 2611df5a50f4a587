# f16 filter kernel sweep at mid sizes (ICP_MFMA16_KERNEL), seeded iterations.
set -u
O=gpurun_out/${1:-r01do}; mkdir -p $O
CFG=${CFG:-C2_bunny C3_horse syn16384 syn65536}
for k in auto pipe unroll plain r4 r8; do
  if [ $k = auto ]; then E=X=1; else E=ICP_MFMA16_KERNEL=$k; fi
  env $E timeout -k 10 300 python tools/configs_probe.py --configs $CFG --variants auto --reps 3 > $O/$k.log 2>&1 || exit 1
done
echo done
