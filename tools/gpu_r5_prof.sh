#!/bin/bash
# Round-5 profiles of the bench command (full library): rocprofv3 kernel stats + the timed window's stats, the PMC
# passes (run_gpu.sh pmc), the GPU suite and smoke(). Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in ${STEPS:-prof pmc tests smoke}; do
  case $step in
  prof|pmc|smoke) bash run_gpu.sh $step || exit $? ;;
  tests)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/r05_gpu_tests.log 2>&1 || exit $? ;;
  esac
done
exit 0
