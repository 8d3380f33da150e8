#!/bin/bash
# k_csr* loop stamps (tools/libswimsim_stamp.so, built with -DCSR_DIAG_STAMP) on real cascade rows
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r5}
for R in ${ROUNDS:-14 18 22}; do
  for rows in ${ROWS:-65536 8192}; do
    SWIMSIM_LIBRARY=${STAMPLIB:-tools/libswimsim_stamp.so} timeout -k 10 200 python -u tools/csr_stamps.py 65536 $R $rows \
      >> gpurun_out/${TAG}_stamps.jsonl 2>> gpurun_out/${TAG}_stamps.err || exit $?
  done
done
