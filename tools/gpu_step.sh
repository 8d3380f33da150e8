cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/cs_bench_real.py 65536 18 21,22,23 2 > gpurun_out/csr.json 2> gpurun_out/csr.err || exit 1
timeout -k 10 240 python -u tools/cs_bench.py 4100 64,4100 2 0,21 verify > gpurun_out/csq.json 2> gpurun_out/csq.err || exit 1
