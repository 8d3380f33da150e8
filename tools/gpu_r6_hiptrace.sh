#!/bin/bash
# kernel trace + HIP API trace of one quick bench run (host pacing between launches); both CSVs gzipped into
# gpurun_out/p6/, the raw output deleted on the box.
# usage: tools/gpu_r6_hiptrace.sh <tag> <bench.py args...>
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/p6
export TMPDIR=/tmp
tag=$1; shift
d=/tmp/hipt_$tag
rm -rf $d
timeout -k 10 500 rocprofv3 --kernel-trace --hip-trace -d $d -o run --output-format csv -- python3 bench.py "$@" \
  > gpurun_out/p6/$tag.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/p6/$tag.log; [ $rc -eq 0 ] || exit $rc
kt=$(ls $d/*/run_kernel_trace.csv $d/run_kernel_trace.csv 2>/dev/null | head -n 1)
ht=$(ls $d/*/run_hip_api_trace.csv $d/run_hip_api_trace.csv 2>/dev/null | head -n 1)
gzip -c "$kt" > gpurun_out/p6/${tag}_ktrace.csv.gz
gzip -c "$ht" > gpurun_out/p6/${tag}_hiptrace.csv.gz
ls -la $d/* >> gpurun_out/p6/$tag.log
rm -rf $d
exit 0
