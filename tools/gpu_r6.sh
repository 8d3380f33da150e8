#!/bin/bash
# round-6 GPU session steps (each under its own time limit; the first failing product step ends the script)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > gpurun_out/r6_gpu_tests.log 2>&1
    rc=$?; echo "pytest rc=$rc" >> gpurun_out/r6_gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 ${BENCH_EXTRA} > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err
    rc=$?; echo "bench rc=$rc" >> gpurun_out/r6_bench.err; [ $rc -eq 0 ] || exit $rc ;;
  benchq)
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ring > gpurun_out/r6_benchq.json 2> gpurun_out/r6_benchq.err
    rc=$?; echo "bench rc=$rc" >> gpurun_out/r6_benchq.err; [ $rc -eq 0 ] || exit $rc ;;
  racy)
    # the perturbed hand-over test against a build with round 5's shared done count: expected to FAIL (exit 1)
    SWIMSIM_LIBRARY=$GRAFT_REPO_ROOT/tools/racy/libswimsim_c3shared.so timeout -k 10 400 python -u -m pytest -v --timeout 300 \
      --timeout-method thread tests/test_cs_ref.py -k "perturbed" > gpurun_out/r6_racy.log 2>&1
    rc=$?; echo "racy pytest rc=$rc (1 expected: the race is caught)" >> gpurun_out/r6_racy.log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
  esac
done
exit 0
