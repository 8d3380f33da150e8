#!/bin/bash
# HBM/L2 fetch bytes (FETCH_SIZE, KB per launch) of the reference-row path's kernels on real cascade rows,
# one rocprofv3 --pmc pass per round (tools/cs_bench_real.py mode 5, 65,536 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5}
for R in ${ROUNDS:-14 18 22}; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_fetch_$R -o run --output-format csv \
    -- python3 tools/cs_bench_real.py 65536 $R 5 1 65536 > gpurun_out/${TAG}_fetch_$R.log 2>&1 || exit $?
done
