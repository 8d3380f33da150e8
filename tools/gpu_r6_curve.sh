#!/bin/bash
# checksum curve on real cascade rows (config 3 at 65,536, rounds 14-22): production choice (mode 0), the reference-row
# path on the main stream (5) and on the side stream with its own buffer set (6, at most 12,288 rows), bit-exact
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/cs && export TMPDIR=/tmp
for R in 14 16 18 20 22; do
  timeout -k 10 200 python -u tools/cs_bench_real.py 65536 $R 0,5,6 2 4096,8192,12288 > gpurun_out/cs/curve_r$R.json 2> gpurun_out/cs/curve_r$R.err || exit 1
  timeout -k 10 200 python -u tools/cs_bench_real.py 65536 $R 0,5 2 16384,65536 > gpurun_out/cs/curve_big_r$R.json 2> gpurun_out/cs/curve_big_r$R.err || exit 1
done
