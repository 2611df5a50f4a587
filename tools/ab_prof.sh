# Same-box rocprofv3 kernel stats of bench.py (C4) for the working tree's library and build_ab/REV:
#   tools/ab_prof.sh TAG REV
set -u
O=gpurun_out/$1; REV=$2
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o bench -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/new.log 2>&1 || exit 1
ICP_AMD_LIB=iterative-closest-point_amd/build_ab/$REV/libicp_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o bench -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases > $O/old.log 2>&1 || exit 1
echo done
