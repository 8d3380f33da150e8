#!/bin/bash
# Diagnostics: run every variants/*.so build (SWIMSIM_LIB) one after another.
#   VAR_MODE=cs (default): checksum microbench (CS_MODES, default 0,2)
#   VAR_MODE=bench       : bench.py --no-cpu-baseline (prints value and kernel_ms)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in variants/*.so; do
  n=$(basename "$v" .so)
  if [ "${VAR_MODE:-cs}" = bench ]; then
    SWIMSIM_LIB=$PWD/$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ring ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || exit $?
    echo "$n $(python3 -c "import json; d=json.load(open('gpurun_out/var_$n.json')); print(d['value'], d['kernel_ms'])")"
  else
    SWIMSIM_LIB=$PWD/$v timeout -k 10 200 python -u tools/cs_bench.py 65536 64,65536 2 ${CS_MODES:-0,2} \
      > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || exit $?
    echo "$n $(cat gpurun_out/var_$n.json)"
  fi
done
