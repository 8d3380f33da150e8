#!/bin/bash
# Round-5 GPU session: parity of the reference-row path (k_csr2), its timing on real cascade rows against round 4's
# k_csr (bench_checksum modes 5 / 6), the bench line, then the whole GPU suite. Each GPU step has its own time
# limit; the script stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5a}
for step in ${STEPS:-csref real bench tests}; do
  case $step in
  csref)
    timeout -k 10 400 python -u -m pytest tests/test_cs_ref.py -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_csref.log 2>&1 || exit $? ;;
  real)
    for R in ${ROUNDS:-14 18 22}; do
      timeout -k 10 240 python -u tools/cs_bench_real.py 65536 $R ${MODES:-5,6} 2 ${ROWS:-65536,8192} \
        > gpurun_out/${TAG}_real_$R.json 2> gpurun_out/${TAG}_real_$R.err || exit $?
    done ;;
  bench)
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_EXTRA:---no-cpu-baseline} \
      > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $? ;;
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > gpurun_out/${TAG}_tests.log 2>&1 || exit $? ;;
  prof)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ring > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
    python3 tools/prof_window.py $(ls gpurun_out/${TAG}_prof/*/run_kernel_trace.csv gpurun_out/${TAG}_prof/run_kernel_trace.csv 2>/dev/null | head -n 1) \
      gpurun_out/${TAG}_prof_window_stats.csv || exit 1 ;;
  esac
done
exit 0
