#!/bin/bash
# Diagnostics: checksum microbench of every variants/*.so build (SWIMSIM_LIB), one after another.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in variants/*.so; do
  n=$(basename "$v" .so)
  SWIMSIM_LIB=$PWD/$v timeout -k 10 200 python -u tools_cs_bench.py 65536 64,65536 2 ${CS_MODES:-0,2} \
    > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || exit $?
  echo "$n $(cat gpurun_out/var_$n.json)"
done
