#!/bin/bash
# rocprofv3 kernel-trace summaries of bench.py commands, kept compact (gpurun copies back <= 64 MiB): per command the
# whole-run kernel stats, the timed-window stats (tools/prof_window.py) and the per-round timeline
# (tools/prof_timeline.py); the raw traces are deleted on the box.
# usage: tools/gpu_r6_prof.sh <tag> <bench.py args...>
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/p6
export TMPDIR=/tmp
tag=$1; shift
d=/tmp/prof_$tag
rm -rf $d
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py "$@" \
  > gpurun_out/p6/$tag.log 2>&1
rc=$?; echo "rocprof rc=$rc" >> gpurun_out/p6/$tag.log; [ $rc -eq 0 ] || exit $rc
tr=$(ls $d/*/run_kernel_trace.csv $d/run_kernel_trace.csv 2>/dev/null | head -n 1)
st=$(ls $d/*/run_kernel_stats.csv $d/run_kernel_stats.csv 2>/dev/null | head -n 1)
cp "$st" gpurun_out/p6/${tag}_kernel_stats.csv
python3 tools/prof_window.py "$tr" gpurun_out/p6/${tag}_window_kernel_stats.csv || exit 1
python3 tools/prof_timeline.py "$tr" gpurun_out/p6/${tag}_round_timeline.txt || exit 1
[ -n "$KEEP_TRACE" ] && gzip -c "$tr" > gpurun_out/p6/${tag}_trace.csv.gz
rm -rf $d
exit 0
