cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 python -u tools/cs_bench.py 65536 64,4096,12288 2 6,33,30,34,35,36,38 verify > gpurun_out/csq.json 2> gpurun_out/csq.err || exit 1
