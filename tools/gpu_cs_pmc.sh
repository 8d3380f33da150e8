#!/bin/bash
# Diagnostics: SQ counters of checksum kernel variants on 64 rows and 65,536 rows (tools/cs_bench.py modes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
MODES=${CS_MODES:-21,22,23}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/cs_pmc1 -o run --output-format csv -- python3 tools/cs_bench.py 65536 64,65536 1 $MODES > gpurun_out/cs_pmc1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM --kernel-trace -d gpurun_out/cs_pmc2 -o run --output-format csv -- python3 tools/cs_bench.py 65536 64,65536 1 $MODES > gpurun_out/cs_pmc2.log 2>&1 || exit 1
