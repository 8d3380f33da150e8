cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 python -u tools/cs_bench.py 65536 64,6208,12288 2 6,30,33 verify > gpurun_out/csq.json 2> gpurun_out/csq.err || exit 1
