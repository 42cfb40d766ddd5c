#!/bin/bash
# LDS bank-conflict scan of the config-5 DQN kernels (acting + update) and the config-3 A3C kernels:
# one --pmc pass each, summarised per kernel by tools/pmc_by_kernel.py.
# usage: bash tools/gpurun/pmc_lds_scan.sh OUTDIR
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES"
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $OUT/dqn -o pmc -- python3 tools/prof_dqn.py 2 > $OUT/dqn.log 2>&1 \
&& timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $OUT/a3c -o pmc -- python3 tools/prof_a3c.py > $OUT/a3c.log 2>&1 \
&& python3 tools/pmc_by_kernel.py $OUT/dqn > $OUT/dqn.txt && python3 tools/pmc_by_kernel.py $OUT/a3c > $OUT/a3c.txt \
&& head -25 $OUT/dqn.txt && head -25 $OUT/a3c.txt
