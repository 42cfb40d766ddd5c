#!/bin/bash
# k_cnn_train kernel A/B with ONE PROCESS PER LIBRARY (in-process library A/Bs carry a few-% systematic
# error: profiles/r05/a3c/train/fence_mask_vmem_ab.txt, sessions 8-9): tools/exp_train.py on the
# trainer's segment-weight instance, libraries alternated over N rounds (order reversed every other
# round). Put the same library under two names to get an A/A control.
# usage: N=4 bash tools/gpurun/train_ab.sh OUT lib.so [lib.so ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
LIBS=("$@")
for i in $(seq ${N:-4}); do
  if [ $((i % 2)) -eq 0 ]; then ORDER=$(printf '%s\n' "${LIBS[@]}" | tac); else ORDER=$(printf '%s\n' "${LIBS[@]}"); fi
  for L in $ORDER; do
    R48_EXP_SEG=1 timeout -k 10 300 python -u tools/exp_train.py 16777216 $L 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
  done
done
cat $O/timing.txt
