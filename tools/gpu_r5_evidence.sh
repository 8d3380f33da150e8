#!/bin/bash
# Round-5 evidence (full library build): the reference-row path on real cascade rows against the production kernels
# (rounds 14-22, shard sizes 65,536 / 16,384 / 8,192 rows), the bench line with its CPU baseline, the 100-round line.
# Each GPU step has its own time limit; the script stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in ${STEPS:-curve bench bench100}; do
  case $step in
  curve)
    for R in ${ROUNDS:-14 16 18 20 22}; do
      timeout -k 10 240 python -u tools/cs_bench_real.py 65536 $R ${MODES:-0,5} 3 ${ROWS:-65536,16384,8192} \
        > gpurun_out/r05_curve_$R.json 2> gpurun_out/r05_curve_$R.err || exit $?
    done ;;
  bench)
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || exit $? ;;
  bench100)
    timeout -k 10 600 python -u bench.py --steps 100 --warmup 0 --no-cpu-baseline > gpurun_out/r05_bench_s100.json \
      2> gpurun_out/r05_bench_s100.err || exit $? ;;
  esac
done
exit 0
