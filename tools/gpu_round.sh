#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script
# (pytest exit 1 = test failures is not a fault, the script goes on to measure).
#   usage: tools/gpu_round.sh TAG [steps...]   steps: test smoke bench prof pmc cli
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift || true
STEPS=${*:-"test smoke bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() { # exit codes that mean the GPU (or the process) died
    case "$1" in 124|137|134|139|-6|-11) return 0 ;; *) return 1 ;; esac
}

run() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -n 25 "$OUT/$name.log"
    if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
    return 0
}

for s in $STEPS; do
    case $s in
    test)  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread --durations=15 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_mfma) run bench_mfma 300 python bench.py --variant mfma --no-cpu-baseline --no-cow ;;
    bench_mfma16) run bench_mfma16 300 python bench.py --variant mfma16 --no-cpu-baseline --no-cow ;;
    bench_valu) run bench_valu 300 python bench.py --variant valu --no-cpu-baseline --no-cow ;;
    bench_fp64) run bench_fp64 300 python bench.py --nn fp64 --steps 5 --warmup 1 --no-cpu-baseline --no-cow ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
               python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases ;;
    profv) for v in ${PROFV:-mfma16 valu}; do
               run rocprof_$v 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o bench -- \
                   python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cow --variant $v; done ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc1" -o fetch -- \
               python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cow --no-cases &&
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc2" -o write -- \
               python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cow --no-cases ;;
    sq)    for v in ${SQV:-mfma valu}; do
               run sq1_$v 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE \
                   --output-format csv -d "$OUT/sq1_$v" -o sq -- python3 tools/nn_probe.py --variant $v --reps 1
               run sq2_$v 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INST_CYCLES_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
                   --output-format csv -d "$OUT/sq2_$v" -o sq -- python3 tools/nn_probe.py --variant $v --reps 1
           done ;;
    sqb)   run sqb1 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE \
               --output-format csv -d "$OUT/sqb1" -o sq -- python3 tools/bundle_probe.py --steps 5 --variants bundle &&
           run sqb2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INST_CYCLES_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
               --output-format csv -d "$OUT/sqb2" -o sq -- python3 tools/bundle_probe.py --steps 5 --variants bundle ;;
    probe) for v in mfma16 mfma valu; do run probe_$v 300 python3 tools/nn_probe.py --variant $v; done ;;
    abpipe) for ld in plain pipe unroll r4 r8; do ICP_MFMA16_KERNEL=$ld run abp_${ld} 300 python3 tools/nn_probe.py --variant mfma16 --icp 12; done ;;
    test16k) for ld in ${K16:-unroll r4}; do
               ICP_MFMA16_KERNEL=$ld run pytest_gpu_$ld 900 python -m pytest tests -m gpu -q -rf -k "mfma16 or grid or sharded or parity" || exit 1
             done ;;
    test16plain) ICP_MFMA16_KERNEL=plain run pytest_gpu_plain 900 python -m pytest tests -m gpu -q -rf -k "mfma16 or grid or sharded" ;;
    dist2) ICP_BENCH_HOST_REDUCE=1 run bench_dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
               --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 ;;
    profcow) COW=$(python3 -c 'import sys; sys.path.insert(0, "tests"); import datasets; print(datasets.path("cow_ref"), datasets.path("cow_tr1"))')
           set -- $COW
           run rocprof_cow 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cow" -o cow -- \
               ./iterative-closest-point_amd/build/icp-bench --ref "$1" --scene "$2" --min-time 0.3 --only opti_gpu_loop ;;
    profcowapi) COW=$(python3 -c 'import sys; sys.path.insert(0, "tests"); import datasets; print(datasets.path("cow_ref"), datasets.path("cow_tr1"))')
           set -- $COW
           run rocprof_cowapi 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/prof_cowapi" -o cow -- \
               ./iterative-closest-point_amd/build/icp-bench --ref "$1" --scene "$2" --min-time 0.1 --only opti_gpu_loop ;;
    sqseed) run sqs1 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE \
                --output-format csv -d "$OUT/sqs1" -o sq -- python3 tools/nn_probe.py --variant mfma16 --icp 4 &&
            run sqs2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE \
                --output-format csv -d "$OUT/sqs2" -o sq -- python3 tools/nn_probe.py --variant mfma16 --icp 4 ;;
    cfg16) for c in 21 22 24 41 42; do ICP_MFMA16_CFG=$c run probe16_$c 300 python3 tools/nn_probe.py --variant mfma16; done ;;
    c5pmc) # rank 0's shard of the 8-way C5 (1-rank RCCL): kernel trace + FETCH / WRITE passes
           run rocprof_c5shard 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5shard" -o c5shard -- \
               python3 tools/shard_probe.py --n 8388608 --worlds 8 --steps 10 --warmup 2 &&
           run pmc_c5shard_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_c5shard1" -o fetch -- \
               python3 tools/shard_probe.py --n 8388608 --worlds 8 --steps 4 --warmup 8 &&
           run pmc_c5shard_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_c5shard2" -o write -- \
               python3 tools/shard_probe.py --n 8388608 --worlds 8 --steps 4 --warmup 8 ;;
    c5dist8) # the 8-rank C5 flow rehearsed on one GPU (8 processes, sums through gloo)
           ICP_BENCH_HOST_REDUCE=1 run bench_c5_dist8 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
               --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --points 8388608 --steps 10 --warmup 2 \
               --no-cpu-baseline --no-cow --no-cases ;;
    shard) run shard_c4 600 python tools/shard_probe.py --worlds 1 2 4 8 &&
           run shard_c5 600 python tools/shard_probe.py --n 8388608 --worlds 8 --steps 5 --warmup 2 ;;
    profshard) run rocprof_shard8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_shard8" -o shard -- \
               python3 tools/shard_probe.py --worlds 8 --steps 20 ;;
    rounds) for r in 1 2 4 1 2 4; do ICP_NN_MIN_ROUNDS=$r ICP_DEBUG_PLAN=1 run rounds_$r 300 python tools/shard_probe.py --worlds 8 4 --steps 20 || exit 1; done ;;
    stride) for r in 1 1000 1 1000; do ICP_NN_TIMING_STRIDE=$r run stride_$r 300 python tools/shard_probe.py --worlds 8 1 --steps 20 || exit 1; cat $OUT/stride_$r.log >> $OUT/stride_all.log; done ;;
    ab) # AB_REV=<rev built by tools/build_ab.sh>: alternate the working tree's library and that one
        for k in 1 2; do
            run ab_new_$k 300 python tools/shard_probe.py --worlds 1 8 --steps 20 || exit 1
            ICP_AMD_LIB=iterative-closest-point_amd/build_ab/$AB_REV/libicp_hip.so run ab_old_$k 300 python tools/shard_probe.py --worlds 1 8 --steps 20 || exit 1
        done ;;
    gridg) for g in 1 4 16 1 4 16; do ICP_GRID_GROUP=$g run gridg_$g 300 python tools/shard_probe.py --variant grid --worlds 1 8 --steps 30 || exit 1; cat $OUT/gridg_$g.log >> $OUT/gridg_all_$g.log; done ;;
    gridr) for g in 4 16 4 16; do ICP_GRID_RGROUP=$g run gridr_$g 300 python tools/shard_probe.py --worlds 1 8 --steps 20 || exit 1; cat $OUT/gridr_$g.log >> $OUT/gridr_all_$g.log; done ;;
    cases) COW=$(python3 -c 'import sys; sys.path.insert(0, "tests"); import datasets; print(datasets.path("cow_ref"), datasets.path("cow_tr1"))')
           set -- $COW
           run cases 300 ./iterative-closest-point_amd/build/icp-bench --ref "$1" --scene "$2" --min-time 0.3 ;;
    fin16) for g in 1 4 8 1 4 8; do ICP_FIN16_LANES=$g run fin16_$g 300 python tools/shard_probe.py --worlds 8 1 --steps 20 || exit 1; cat $OUT/fin16_$g.log >> $OUT/fin16_all_$g.log; done ;;
    profhorse) run rocprof_horse 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_horse" -o horse -- \
               python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 3 ;;
    gridrh) for g in 16 64 4 16 64; do ICP_GRID_RGROUP=$g run gridrh_$g 300 python tools/configs_probe.py --configs C3_horse C2_bunny --variants auto || exit 1; cat $OUT/gridrh_$g.log >> $OUT/gridrh_all_$g.log; done ;;
    gridr64) for g in 16 64 16 64; do ICP_GRID_RGROUP=$g run gridr64_$g 300 python tools/shard_probe.py --worlds 1 8 --steps 20 || exit 1; cat $OUT/gridr64_$g.log >> $OUT/gridr64_all_$g.log; done ;;
    gseed) for v in 0 1 0 1; do ICP_GRID_SEED=$v run gseed_$v 300 python3 tools/nn_probe.py --variant mfma16 --reps 3 || exit 1; cat $OUT/gseed_$v.log >> $OUT/gseed_all_$v.log; done ;;
    configs) run configs 300 python tools/configs_probe.py ;;
    calib) run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib1" -o fetch -- tools/hbm_calib &&
           run calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib2" -o write -- tools/hbm_calib ;;
    test_new) run pytest_new 900 python -u -m pytest tests/test_gpu_c4c5.py tests/test_gpu_boundary.py tests/test_gpu_cert_stress.py \
               tests/test_gpu_grid.py -m gpu -v -rf --timeout 300 --timeout-method thread --durations=15 ;;
    test_pers) run pytest_pers 300 python -u -m pytest tests/test_gpu_persistent.py -m gpu -v -rf --timeout 120 --timeout-method thread --durations=10 ;;
    cowab) for m in launches persistent launches persistent; do ICP_RUN_MODE=$m run cowab_$m 300 ./iterative-closest-point_amd/build/icp-bench \
               --ref "$(python3 -c 'import sys; sys.path.insert(0, "tests"); import datasets; print(datasets.path("cow_ref"))')" \
               --scene "$(python3 -c 'import sys; sys.path.insert(0, "tests"); import datasets; print(datasets.path("cow_tr1"))')" \
               --min-time 0.3 --only opti_gpu_loop || exit 1; cat $OUT/cowab_$m.log >> $OUT/cowab_all_$m.log; done ;;
    midab) run midab 300 python tools/configs_probe.py --configs C2_bunny C3_horse syn20000 --variants auto loop --reps 5 &&
           ICP_PERSIST_STAMPS=1 run midstamps 120 python tools/configs_probe.py --configs C3_horse C2_bunny --variants auto --reps 1 ;;
    testrccl) run pytest_rccl 300 python -m pytest tests/test_gpu_sharded.py -m gpu -q -rf -k rccl ;;
    cli)   run cli 300 bash -c "cd $OUT && ../../iterative-closest-point_amd/build/icp-gpu \
               \$(python3 -c 'import sys;sys.path.insert(0,\"../../tests\");import datasets;print(datasets.path(\"cow_ref\"),datasets.path(\"cow_tr1\"))') 20" ;;
    test_c5) run pytest_c5 900 python -u -m pytest tests/test_gpu_c5_sharded.py tests/test_gpu_boundary.py -m gpu -v -rf \
               --timeout 600 --timeout-method thread --durations=10 ;;
    c3hbm) run c3_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3_trace" -o c3 -- \
               python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 1 &&
           run c3_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c3_pmc1" -o fetch -- \
               python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 1 &&
           run c3_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c3_pmc2" -o write -- \
               python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 1 &&
           ICP_PERSIST_STAMPS=1 run c3_stamps 120 python3 tools/configs_probe.py --configs C3_horse --variants auto --reps 1 ;;
    gridhbm) run grid_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/grid_trace" -o grid -- \
               python3 bench.py --variant grid --steps 10 --warmup 2 --no-cpu-baseline --no-cow --no-cases &&
           run grid_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/grid_pmc1" -o fetch -- \
               python3 bench.py --variant grid --steps 3 --warmup 1 --no-cpu-baseline --no-cow --no-cases &&
           run grid_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/grid_pmc2" -o write -- \
               python3 bench.py --variant grid --steps 3 --warmup 1 --no-cpu-baseline --no-cow --no-cases ;;
    bprobe) run bprobe 600 python3 tools/bundle_probe.py --steps 10 --variants mfma16 bundle &&
            run bprobe8 300 python3 tools/bundle_probe.py --steps 10 --shard 8 --variants mfma16 bundle ;;
    test_bundle) run pytest_bundle 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_c4c5.py -m gpu -x -v -rf \
               --timeout 300 --timeout-method thread --durations=10 -k "bundle or c4 or split" ;;
    bsweep) for r in 4 2 1; do
               ICP_NN_MIN_ROUNDS=$r ICP_DEBUG_PLAN=1 run bsweep_r$r 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               ICP_NN_MIN_ROUNDS=$r ICP_DEBUG_PLAN=1 run bsweep8_r$r 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
             done
             run bsweep2 300 python3 tools/bundle_probe.py --steps 20 --shard 2 --variants bundle &&
             run bsweep4 300 python3 tools/bundle_probe.py --steps 20 --shard 4 --variants bundle ;;
    bmid) for n in 16384 40000 65536 262144; do run bmid_$n 300 python3 tools/bundle_probe.py --n $n --steps 20 --variants mfma16 bundle || exit 1; done ;;
    bgab) for g in 1 0 1 0; do
              ICP_BUNDLE_GROUP=$g run bgab_$g 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
              ICP_BUNDLE_GROUP=$g run bgab8_$g 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
              cat $OUT/bgab_$g.log $OUT/bgab8_$g.log >> $OUT/bgab_all_$g.log
          done ;;
    bv2) for cfg in "ICP_BUNDLE_KERNEL=2 ICP_BUNDLE_QG=8" "ICP_BUNDLE_KERNEL=2 ICP_BUNDLE_QG=4" "ICP_BUNDLE_KERNEL=1" "ICP_BUNDLE_KERNEL=2 ICP_BUNDLE_QG=8"; do
             tag=$(echo $cfg | tr -d ' =_' | tr 'A-Z' 'a-z')
             env $cfg timeout -k 10 300 python3 tools/bundle_probe.py --steps 20 --variants bundle >> $OUT/bv2_$tag.log 2>&1 || exit 1
             env $cfg timeout -k 10 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle >> $OUT/bv2_$tag.log 2>&1 || exit 1
             env $cfg timeout -k 10 300 python3 tools/bundle_probe.py --n 8388608 --shard 8 --steps 5 --warmup 1 --variants bundle >> $OUT/bv2_$tag.log 2>&1 || exit 1
             echo "== bv2 $cfg done" | tee -a $OUT/steps.log
           done ;;
    bprof) run bprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bprof" -o c4 -- \
               python3 tools/bundle_probe.py --steps 20 --variants bundle &&
           run bprof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bprof8" -o s8 -- \
               python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle ;;
    bsplit) for sp in 1 2 3 4 6 8; do
               ICP_BUNDLE_SPLITS=$sp run bsplit_$sp 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             done
             for sp in 6 12 18 24; do
               ICP_BUNDLE_SPLITS=$sp run bsplit8_$sp 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
             done
             for sp in 2 3 4; do
               ICP_BUNDLE_QG=4 ICP_BUNDLE_SPLITS=$sp run bsplitq4_$sp 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             done ;;
    splitdiag) run splitdiag 60 ./tools/split_probe ;;
    test_tail) run pytest_tail 300 python -u -m pytest tests/test_gpu_persistent.py -m gpu -x -v -rf --timeout 120 \
               --timeout-method thread -k "abort" ;;
    test_cert) run pytest_cert 600 python -u -m pytest tests/test_gpu_cert_stress.py tests/test_gpu_persistent.py -m gpu -x -v -rf \
               --timeout 300 --timeout-method thread -k "cert or scale_fuzz" ;;
    bpb) for pb in 4 8 4 8; do
           ICP_BUNDLE_PB=$pb run bpb_$pb 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
           ICP_BUNDLE_PB=$pb run bpb8_$pb 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
           cat $OUT/bpb_$pb.log $OUT/bpb8_$pb.log >> $OUT/bpb_all_$pb.log
         done ;;
    bilv) for il in 1 0 1 0; do
            ICP_BUNDLE_ILV=$il run bilv_$il 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
            ICP_BUNDLE_ILV=$il run bilv8_$il 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
            cat $OUT/bilv_$il.log $OUT/bilv8_$il.log >> $OUT/bilv_all_$il.log
          done
          for sm in 64 128; do
            ICP_BUNDLE_SMAX=$sm run bsm8_$sm 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
          done ;;
    btask3) run bdef 300 python3 tools/bundle_probe.py --steps 20 --variants bundle mfma16 || exit 1
            run bdef8 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
            run bdef4 300 python3 tools/bundle_probe.py --steps 20 --shard 4 --variants bundle || exit 1
            run bdef2 300 python3 tools/bundle_probe.py --steps 20 --shard 2 --variants bundle || exit 1 ;;
    btask2) for cfg in "32 16" "64 16" "128 16" "32 32" "64 32" "16 32"; do
             set -- $cfg
             ICP_BUNDLE_CH=$1 ICP_BUNDLE_SMAX=$2 run bt_$1_$2 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             ICP_BUNDLE_CH=$1 ICP_BUNDLE_SMAX=$2 run bt8_$1_$2 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
           done ;;
    btask) run bdef 300 python3 tools/bundle_probe.py --steps 20 --variants bundle mfma16 || exit 1
           run bdef8 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
           for ch in 4 16 32; do
             ICP_BUNDLE_CH=$ch run bch_$ch 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             ICP_BUNDLE_CH=$ch run bch8_$ch 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
           done
           for sm in 8 32; do
             ICP_BUNDLE_SMAX=$sm run bsm_$sm 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             ICP_BUNDLE_SMAX=$sm run bsm8_$sm 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
           done
           ICP_BUNDLE_QG=4 run bq4 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1 ;;
    bsplit3) run bdef 300 python3 tools/bundle_probe.py --steps 20 --variants bundle mfma16 || exit 1
             run bdef8 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
             ICP_BUNDLE_CAND=0 run bnocand 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             for sp in 1 2 4 8; do
               ICP_BUNDLE_SPLITS=$sp run bsplit_$sp 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             done
             for sp in 4 8 24; do
               ICP_BUNDLE_SPLITS=$sp run bsplit8_$sp 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
             done
             for sp in 1 2 4; do
               ICP_BUNDLE_QG=4 ICP_BUNDLE_SPLITS=$sp run bsplitq4_$sp 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             done ;;
    bsplit2) run bdef 300 python3 tools/bundle_probe.py --steps 20 --variants bundle mfma16 || exit 1
             run bdef8 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
             for sp in 6 12 16; do
               ICP_BUNDLE_SPLITS=$sp run bsplit_$sp 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             done
             for sp in 24 48; do
               ICP_BUNDLE_SPLITS=$sp run bsplit8_$sp 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
             done
             for sp in 8 16; do
               ICP_BUNDLE_QG=4 ICP_BUNDLE_SPLITS=$sp run bsplitq4_$sp 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
             done ;;
    sceneab) for o in 1 0 1 0; do
               ICP_SCENE_ORDER=$o run sceneab_$o 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               cat $OUT/sceneab_$o.log >> $OUT/sceneab_all_$o.log
               ICP_SCENE_ORDER=$o run sceneab8_$o 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
               cat $OUT/sceneab8_$o.log >> $OUT/sceneab_all_$o.log
               ICP_SCENE_ORDER=$o run sceneabg_$o 300 python3 bench.py --variant grid --steps 20 --no-cpu-baseline --no-cow --no-cases || exit 1
               cat $OUT/sceneabg_$o.log >> $OUT/sceneab_all_$o.log
             done ;;
    recab) for o in 1 0 1 0; do
               ICP_TRANSFORM_RECORDS=$o run recab_$o 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               cat $OUT/recab_$o.log >> $OUT/recab_all_$o.log
               ICP_TRANSFORM_RECORDS=$o run recab8_$o 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
               cat $OUT/recab8_$o.log >> $OUT/recab_all_$o.log
             done ;;
    pmcsq) run pmcsq1 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
               --output-format csv -d "$OUT/pmcsq1" -o sq -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cow --no-cases &&
           run pmcsq2 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE \
               --output-format csv -d "$OUT/pmcsq2" -o sq -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cow --no-cases ;;
    percu) for pc in 2 3 4 2 3 4; do
               ICP_BUNDLE_PER_CU=$pc ICP_DEBUG_PLAN=1 run percu_$pc 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               cat $OUT/percu_$pc.log >> $OUT/percu_all_$pc.log
               ICP_BUNDLE_PER_CU=$pc run percu8_$pc 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
               cat $OUT/percu8_$pc.log >> $OUT/percu_all_$pc.log
             done ;;
    libab) # LIBS="name ..." (iterative-closest-point_amd/build_ab/<name>/libicp_hip.so; "tree" = the working tree's)
           for k in 1 2; do
             for L in ${LIBS:-tree}; do
               lib=""; [ "$L" != tree ] && lib=iterative-closest-point_amd/build_ab/$L/libicp_hip.so
               ICP_AMD_LIB=$lib run libab_${L}_$k 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               cat $OUT/libab_${L}_$k.log >> $OUT/libab_all_$L.log
               ICP_AMD_LIB=$lib run libab8_${L}_$k 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
               cat $OUT/libab8_${L}_$k.log >> $OUT/libab_all_$L.log
             done
           done ;;
    qg4) for k in 1 2; do
           ICP_BUNDLE_QG=4 run qg4_$k 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
           ICP_BUNDLE_QG=4 run qg48_$k 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
           cat $OUT/qg4_$k.log $OUT/qg48_$k.log >> $OUT/qg4_all.log
         done ;;
    localab) for o in 1 0 1 0; do
               ICP_BUNDLE_LOCAL=$o run localab_$o 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               ICP_BUNDLE_LOCAL=$o run localab8_$o 300 python3 tools/bundle_probe.py --steps 20 --shard 8 --variants bundle || exit 1
               cat $OUT/localab_$o.log $OUT/localab8_$o.log >> $OUT/localab_all_$o.log
             done ;;
    finab) for k in 1 2; do
             for r in 8 4 2 1; do
               ICP_FIN16_ROUNDS=$r run finab_${r}_$k 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
               cat $OUT/finab_${r}_$k.log >> $OUT/finab_all_$r.log
             done
           done ;;
    rbab) for k in 1 2; do
            for b in 4096 1024 256; do
              ICP_GRID_RBLOCKS=$b run rbab_${b}_$k 300 python3 tools/bundle_probe.py --steps 20 --variants bundle || exit 1
              cat $OUT/rbab_${b}_$k.log >> $OUT/rbab_all_$b.log
            done
          done ;;
    midth) for k in 1 2; do
             for t in 512 768 1024; do
               ICP_MID_THREADS=$t run midth_${t}_$k 300 python3 tools/configs_probe.py --configs C2_bunny C3_horse --variants auto --reps 5 || exit 1
               cat $OUT/midth_${t}_$k.log >> $OUT/midth_all_$t.log
             done
           done ;;
    test_midth) for t in ${MIDTH:-768 1024}; do
               ICP_MID_THREADS=$t run pytest_midth_$t 300 python -u -m pytest tests/test_gpu_persistent.py tests/test_gpu_cpu_rule.py -m gpu -x -q -rf \
                   --timeout 120 --timeout-method thread || exit 1
             done ;;
    momab) for k in 1 2; do
             for b in 1 4 2; do
               ICP_MOM_BATCH=$b run momab_${b}_$k 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/momab_${b}_$k" -o c4 -- \
                   python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cow --no-cases || exit 1
             done
           done ;;
    shardab) for k in 1 2; do
               for L in ${LIBS:-tree}; do
                 lib=""; [ "$L" != tree ] && lib=iterative-closest-point_amd/build_ab/$L/libicp_hip.so
                 ICP_AMD_LIB=$lib run shardab_${L}_$k 300 python tools/shard_probe.py --worlds 1 8 --steps 20 || exit 1
                 cat $OUT/shardab_${L}_$k.log >> $OUT/shardab_all_$L.log
               done
             done ;;
    c5shard) run c5shard 300 python tools/shard_probe.py --n 8388608 --worlds 8 --steps 5 --warmup 2 ;;
    fuseab) for k in 1 2; do
              for f in 1 0; do
                ICP_BUNDLE_FUSE_TASKS=$f run fuseab_${f}_$k 300 python tools/shard_probe.py --worlds 1 8 --steps 20 || exit 1
                cat $OUT/fuseab_${f}_$k.log >> $OUT/fuseab_all_$f.log
                ICP_BUNDLE_FUSE_TASKS=$f run fusebench_${f}_$k 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-cow --no-cases || exit 1
                cat $OUT/fusebench_${f}_$k.log >> $OUT/fuseab_all_$f.log
              done
            done ;;
    finw8) for k in 1 2; do
             for r in 1 2 4; do
               ICP_FIN16_ROUNDS=$r run finw8_${r}_$k 300 python tools/shard_probe.py --worlds 8 4 --steps 20 || exit 1
               cat $OUT/finw8_${r}_$k.log >> $OUT/finw8_all_$r.log
             done
           done ;;
    strideab) for k in 1 2; do
                for r in 8 1; do
                  ICP_NN_TIMING_STRIDE=$r run strideab_${r}_$k 300 python tools/shard_probe.py --worlds 1 8 --steps 40 || exit 1
                  cat $OUT/strideab_${r}_$k.log >> $OUT/strideab_all_$r.log
                  ICP_NN_TIMING_STRIDE=$r run stridebench_${r}_$k 300 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-cow --no-cases || exit 1
                  cat $OUT/stridebench_${r}_$k.log >> $OUT/strideab_all_$r.log
                done
              done ;;
    test_bf) ICP_AMD_LIB=iterative-closest-point_amd/build_ab/bf/libicp_hip.so run pytest_bf 600 python -u -m pytest \
               tests/test_gpu_c4c5.py tests/test_gpu_parity.py tests/test_gpu_cert_stress.py -m gpu -x -q -rf \
               --timeout 300 --timeout-method thread ;;
    *) echo "unknown step $s" ;;
    esac
done
echo "done: $STEPS"
