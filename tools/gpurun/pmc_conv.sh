#!/bin/bash
# SQ / HBM counters of the config-5 update convolutions (separate --pmc passes, kernel dispatches
# only), then the kernel breakdown of one update. usage: bash tools/gpurun/pmc_conv.sh [out dir]
set -o pipefail
OUT=${1:-gpurun_out/pmc_conv}
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 tools/exp_conv.py 65536"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $OUT/p1 -o pmc -- $P > $OUT/p1.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o pmc -- $P > $OUT/p2.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o pmc -- $P > $OUT/f.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o pmc -- $P > $OUT/w.log 2>&1 \
&& for k in "k_conv_wgradILi64" "k_conv3x3ILi2" "k_conv_wgradILi32" "k_conv3x3ILi1"; do \
     for g in 65536 131072; do python3 tools/pmc_summary.py $k $g $OUT/p1 $OUT/p2 $OUT/f $OUT/w > $OUT/$k.$g.json; done; done \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o dqn -- python3 tools/prof_dqn.py > $OUT/prof_dqn.log 2>&1 && tail -2 $OUT/prof_dqn.log
