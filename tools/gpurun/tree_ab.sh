#!/bin/bash
# Timing A/B of two code trees (Python + library together: for changes that alter a packed layout,
# where one library cannot run under the other tree's packer): the current tree vs OLD (a copy of an
# earlier tree with its own built library, e.g. `git archive <rev> rein48_amd tools bench.py oracle`),
# one process per arm, alternated over N rounds (order reversed every other round).
# usage: N=4 bash tools/gpurun/tree_ab.sh OUT OLD_DIR "python command run from each tree's root"
set -o pipefail
O=gpurun_out/$1; OLD=$2; CMD=$3; mkdir -p $O
for i in $(seq ${N:-4}); do
  if [ $((i % 2)) -eq 0 ]; then ARMS="new old"; else ARMS="old new"; fi
  for a in $ARMS; do
    if [ $a = old ]; then D=$OLD; else D=.; fi
    (cd $D && timeout -k 10 300 bash -c "$CMD") 2>&1 | grep -v amdgpu.ids | sed "s/^/$a /" >> $O/timing.txt || exit 1
  done
done
cat $O/timing.txt
