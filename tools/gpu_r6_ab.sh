#!/bin/bash
# A/B of an engine environment setting: quick bench lines alternating the values, each under its own time limit; the
# first failing run ends the script.
# usage: tools/gpu_r6_ab.sh <VAR> <value> [<value> ...]   (value "def" = the variable unset)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
var=$1; shift
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = def ]; then unset "$var"; else export "$var=$v"; fi
  tag=$(basename "$v" | tr -c 'A-Za-z0-9_.=-\n' '_')
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ring ${BENCH_EXTRA} \
    > gpurun_out/ab/b${i}_$tag.json 2> gpurun_out/ab/b${i}_$tag.err
  rc=$?; echo "bench rc=$rc" >> gpurun_out/ab/b${i}_$tag.err; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'])" \
    gpurun_out/ab/b${i}_$tag.json "$var=$v"
done
exit 0
