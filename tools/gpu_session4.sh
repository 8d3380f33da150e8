#!/bin/bash
# Round-4 GPU session (diagnostics): op costs, reference-chain microbench, checksum kernel variants on real cascade
# rows, then the GPU test suite. Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/opcost > gpurun_out/opcost.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest exit $?"
