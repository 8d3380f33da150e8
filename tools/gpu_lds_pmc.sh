#!/bin/bash
# LDS bank conflicts and LDS busy cycles of the reference-row path's kernels on real cascade rows (rounds 14 and 18),
# one rocprofv3 --pmc pass per round (tools/cs_bench_real.py mode 5, 65,536 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5}
for R in ${ROUNDS:-14 18}; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-trace -d gpurun_out/${TAG}_ldspmc_$R -o run --output-format csv \
    -- python3 tools/cs_bench_real.py 65536 $R 5 1 65536 > gpurun_out/${TAG}_ldspmc_$R.log 2>&1 || exit $?
done
