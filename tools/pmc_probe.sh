# Counter passes over one kernel of the C4 bench iteration (each pass its own rocprofv3 run,
# within the per-block slot limits), plus the gfx950 counter list.
#   tools/pmc_probe.sh TAG KERNEL_REGEX [extra env assignments, e.g. ICP_GRID_SEEDED=2,2,2]
# A pass that fails on its counter names is reported and the next one runs; a pass that is
# killed, times out or crashes ends the script.
set -u
T=${1:-pmcp}; K=${2:-nn_grid_seeded}; shift 2 || true
O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
rc=$?; [ $rc -ge 124 ] && { echo "counter list rc=$rc"; exit 1; }
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  echo "== pass $i: $pass" | tee -a $O/passes.txt
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-include-regex "$K" --output-format csv -d $O/p$i -o p -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cow --no-cases --no-registration > $O/p$i.log 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a $O/passes.txt
  [ $rc -ge 124 ] && exit 1
done <<'EOF'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum
TA_FLAT_READ_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum
EOF
echo done
