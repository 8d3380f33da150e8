#!/bin/bash
# the reference-row path (bench_checksum mode 5) on real cascade rows with several builds of the library
# (LIBS: tools/libswimsim_*.so names, "prod" = the product library), rounds ROUNDS, rows ROWS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r5}
for lib in ${LIBS:-prod}; do
  for R in ${ROUNDS:-14 18 22}; do
    if [ "$lib" = prod ]; then unset SWIMSIM_LIBRARY; else export SWIMSIM_LIBRARY="tools/libswimsim_$lib.so"; fi
    timeout -k 10 240 python -u tools/cs_bench_real.py 65536 $R ${MODES:-5} 2 ${ROWS:-65536,8192} \
      | tail -n 1 | sed "s/^/{\"lib\": \"$lib\", /; s/^{\"lib\": \"$lib\", {/{\"lib\": \"$lib\", /" >> gpurun_out/${TAG}_variants.jsonl || exit $?
  done
done
