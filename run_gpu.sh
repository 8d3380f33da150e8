#!/bin/bash
# GPU session script: parity tests, then bench; stop at the first failing step
cd "$GRAFT_REPO_ROOT"
mode=${1:-all}
if [ "$mode" = all ] || [ "$mode" = tests ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$mode" = all ] || [ "$mode" = bench ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$mode" = prof ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$mode" = pmc ]; then
  export TMPDIR=/tmp
  SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
  timeout -k 10 300 rocprofv3 --pmc $SQ --kernel-trace -d gpurun_out/pmc_sq -o run --output-format csv -- python3 tools_cs_bench.py 65536 16384 1 > gpurun_out/pmc_sq.log 2>&1
  rc=$?; echo "pmc sq rc=$rc" >> gpurun_out/pmc_sq.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 30 > gpurun_out/pmc_fetch.log 2>&1
  rc=$?; echo "pmc fetch rc=$rc" >> gpurun_out/pmc_fetch.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 30 > gpurun_out/pmc_write.log 2>&1
  rc=$?; echo "pmc write rc=$rc" >> gpurun_out/pmc_write.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
