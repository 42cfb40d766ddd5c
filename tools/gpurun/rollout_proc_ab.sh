#!/bin/bash
# CNN rollout megakernel timing (tools/exp_rollout.py, config-3 size) with ONE library per process,
# libraries alternated over N rounds (order reversed every other round). No parity step: use it for
# timing probes; product candidates go through rollout_ab.sh / cnn_ab.sh.
# usage: N=4 bash tools/gpurun/rollout_proc_ab.sh OUT lib.so [lib.so ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
LIBS=("$@")
for i in $(seq ${N:-4}); do
  if [ $((i % 2)) -eq 0 ]; then ORDER=$(printf '%s\n' "${LIBS[@]}" | tac); else ORDER=$(printf '%s\n' "${LIBS[@]}"); fi
  for L in $ORDER; do
    R48_LIB=$L timeout -k 10 300 python -u tools/exp_rollout.py $L 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
  done
done
cat $O/timing.txt
