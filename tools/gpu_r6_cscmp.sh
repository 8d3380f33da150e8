cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/cs && export TMPDIR=/tmp
for R in 14 18 20 22; do
  timeout -k 10 200 python -u tools/cs_bench_real.py 65536 $R 0,5 2 8192,16384,65536 > gpurun_out/cs/sort_r$R.json 2> gpurun_out/cs/sort_r$R.err || exit 1
  CS_TUNING='{"fault_inject": 512}' timeout -k 10 200 python -u tools/cs_bench_real.py 65536 $R 5 2 8192,16384,65536 > gpurun_out/cs/nosort_r$R.json 2> gpurun_out/cs/nosort_r$R.err || exit 1
done
