cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/cs_bench_real.py 65536 18 21,46 3 > gpurun_out/csr.json 2> gpurun_out/csr.err || exit 1
