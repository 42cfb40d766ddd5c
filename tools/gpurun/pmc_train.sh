#!/bin/bash
# SQ counters of k_cnn_train (separate --pmc passes, kernel dispatches only, no trace domains):
# where the wave cycles go. usage: bash tools/gpurun/pmc_train.sh [out dir]
set -o pipefail
OUT=${1:-gpurun_out/pmc_train}
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 tools/prof_train.py 16777216 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $OUT/p1 -o pmc -- $P > $OUT/p1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o pmc -- $P > $OUT/p2.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES SQ_CYCLES SQ_INST_CYCLES_VMEM GRBM_COUNT --output-format csv -d $OUT/p3 -o pmc -- $P > $OUT/p3.log 2>&1 \
&& python3 tools/pmc_summary.py k_cnn_train ${GRID:-65536} $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/summary.json && cat $OUT/summary.json
