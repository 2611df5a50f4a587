# Same-box A/B of the working tree's library against build_ab/REV (tools/build_ab.sh REV):
#   tools/ab_lib.sh TAG REV [configs...]
set -u
O=gpurun_out/$1; REV=$2; shift 2
CFG=${*:-C2_bunny C3_horse syn16384 syn65536}
mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python tools/configs_probe.py --configs $CFG --variants auto --reps 3 >> $O/new.log 2>&1 || exit 1
  ICP_AMD_LIB=iterative-closest-point_amd/build_ab/$REV/libicp_hip.so timeout -k 10 300 python tools/configs_probe.py --configs $CFG --variants auto --reps 3 >> $O/old.log 2>&1 || exit 1
done
echo done
