#!/bin/bash
# SQ counters of k_cnn_train (separate --pmc passes, no trace domains): where the wave cycles go.
set -o pipefail
OUT=gpurun_out/pmc_train
mkdir -p $OUT
export TMPDIR=/tmp
P="python tools/prof_train.py 16777216 3"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $OUT/p1 -o pmc -- $P > $OUT/p1.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o pmc -- $P > $OUT/p2.log 2>&1
