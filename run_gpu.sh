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
exit 0
