#!/bin/bash
# GPU session script: each step under its own time limit; stop at the first failing step.
# usage: run_gpu.sh [tests|smoke|bench|prof|pmc|calib|curve|all ...]   (several modes run in the order given)
# BENCH_ARGS defaults to the driver's round-end command (--steps 20 --warmup 5); prof and pmc profile
# exactly that command, so profiles/ figures and the bench line describe the same workload.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 5}
PROF_ARGS="$BENCH_ARGS --no-cpu-baseline --no-ring"
WL=${WL:-65536:20:5:1}
[ $# -eq 0 ] && set -- all
for mode in "$@"; do
  case $mode in
  tests|all)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > gpurun_out/gpu_tests.log 2>&1
    rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
    ;;&
  smoke|all)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
    ;;&
  bench|all)
    timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
    rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
    ;;&
  prof|all)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
      -- python3 bench.py $PROF_ARGS > gpurun_out/prof.log 2>&1
    rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
    python3 tools/prof_window.py $(ls gpurun_out/prof/*/run_kernel_trace.csv gpurun_out/prof/run_kernel_trace.csv 2>/dev/null | head -n 1) \
      gpurun_out/prof_window_stats.csv || exit 1
    ;;&
  pmc|all)
    # separate passes (a pass holds at most 8 SQ / 4 TCC counters), each cut to the timed rounds (--window)
    i=0
    for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
                "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
                "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      timeout -k 10 -s KILL 400 rocprofv3 --pmc $pass --kernel-trace -d /tmp/pmc_$i -o run \
        --output-format csv -- python3 bench.py $PROF_ARGS > gpurun_out/pmc_$i.log 2>&1
      rc=$?; echo "pmc pass $i ($pass) rc=$rc" >> gpurun_out/pmc_$i.log; [ $rc -eq 0 ] || exit $rc
    done
    dirs=""
    for k in $(seq 1 $i); do dirs="$dirs $(dirname $(ls /tmp/pmc_$k/*/run_counter_collection.csv /tmp/pmc_$k/run_counter_collection.csv 2>/dev/null | head -n 1))"; done
    python3 tools/pmc_summary.py --workload $WL --window gpurun_out/pmc_summary.json $dirs || exit 1
    ;;&
  calib|all)
    timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calib_fetch -o run --output-format csv \
      -- tools/fetch_calib > gpurun_out/calib.json 2> gpurun_out/calib.err || exit 1
    timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/calib_write -o run --output-format csv \
      -- tools/fetch_calib > /dev/null 2>> gpurun_out/calib.err || exit 1
    ;;
  bench2)
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 2 --members 2048 --steps 30 --warmup 10 --host-transport \
      > gpurun_out/bench2.json 2> gpurun_out/bench2.err
    rc=$?; echo "bench2 rc=$rc" >> gpurun_out/bench2.err; [ $rc -eq 0 ] || exit $rc
    ;;
  curve)
    # rows-vs-ms of the production checksum kernels on real cascade rows (config 3 at 65,536, round 18), parity-checked
    timeout -k 10 300 python -u tools/cs_bench_real.py 65536 18 0,1,2 2 2048,4096,6144,8192,10240,12288,16384,24576,32768,49152,65536 \
      > gpurun_out/curve.json 2> gpurun_out/curve.err
    rc=$?; echo "curve rc=$rc" >> gpurun_out/curve.err; [ $rc -eq 0 ] || exit $rc
    ;;
  csbench)
    timeout -k 10 300 python -u tools/cs_bench.py 65536 64,1024,16384,65536 2 ${CS_MODES:-0,1,2} > gpurun_out/csbench.json 2> gpurun_out/csbench.err
    rc=$?; echo "csbench rc=$rc" >> gpurun_out/csbench.err; [ $rc -eq 0 ] || exit $rc
    ;;
  esac
done
exit 0
