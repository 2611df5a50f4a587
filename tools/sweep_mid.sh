# Mid-size launch-shape sweep of the seeded f16 filter (C2 / C3 / synthetic sizes).
set -u
O=gpurun_out/${1:-r01dc}; mkdir -p $O
CFG=${CFG:-C2_bunny C3_horse syn16384 syn32768 syn65536 syn131072}
run() { # name env...
  local name=$1; shift
  env "$@" ICP_DEBUG_PLAN=1 timeout -k 10 300 python tools/configs_probe.py --configs $CFG --variants auto --reps 3 > $O/$name.log 2>&1 || exit 1
}
run auto X=1
run r8 ICP_MFMA16_KERNEL=r8
run rounds2 ICP_NN_MIN_ROUNDS=2
run rounds3 ICP_NN_MIN_ROUNDS=3
run rounds6 ICP_NN_MIN_ROUNDS=6
timeout -k 10 300 python tools/shard_probe.py --worlds 1 8 > $O/shard.log 2>&1 || exit 1
echo done
