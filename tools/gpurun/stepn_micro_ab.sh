#!/bin/bash
# A/B of k_step_n library variants (tools/exp_stepn_ab.py, two processes) after the instruction-rate
# microbenchmark.  usage: bash tools/gpurun/stepn_micro_ab.sh OUT lib.so ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 120 build/instr_rate > $O/instr_rate.txt 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python -u tools/exp_stepn_ab.py "$@" 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1; done
cat $O/ab.txt; tail -8 $O/instr_rate.txt
