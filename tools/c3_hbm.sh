# C3 (horse_ref vs horse_tr1, 50 iterations): rocprofv3 kernel trace + the two PMC passes for
# per-kernel HBM bytes (BASELINE config C3's "rocprof HBM-GB/s capture").
set -u
O=gpurun_out/${1:-r01dp}; mkdir -p $O; export TMPDIR=/tmp
P="python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c3 -- $P > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc1 -o fetch -- $P > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc2 -o write -- $P > $O/pmc2.log 2>&1 || exit 1
echo done
