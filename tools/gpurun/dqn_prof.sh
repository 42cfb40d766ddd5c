#!/bin/bash
# GPU job: kernel trace of 5 config-5 updates (tools/prof_dqn.py) and its per-update breakdown.
# usage: bash tools/gpurun/dqn_prof.sh [out dir]
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/dqn_prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o dqn -- python3 tools/prof_dqn.py 5 > $O/prof_dqn.log 2>&1; rc=$?; grep "ms" $O/prof_dqn.log; [ $rc -eq 0 ] \
&& python3 tools/dqn_breakdown.py $O/prof/dqn_kernel_trace.csv 6 > $O/breakdown.txt && head -40 $O/breakdown.txt \
&& timeout -k 10 120 python3 tools/prof_dqn.py 10 > $O/update_noprof.txt 2>&1 && cat $O/update_noprof.txt
