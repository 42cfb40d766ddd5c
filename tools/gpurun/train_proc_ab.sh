#!/bin/bash
# k_cnn_train variants: the fused-update parity tests on every variant library, then
# tools/gpurun/train_ab.sh (one process per library, alternated).  usage: bash tools/gpurun/train_proc_ab.sh OUT lib.so ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for L in "$@"; do
  R48_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_a3c_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused_cnn_update or per_board_weights or trainer_fused_update" > $O/pytest_$(basename $L .so).log 2>&1; rc=$?
  echo "$(basename $L): $(tail -1 $O/pytest_$(basename $L .so).log)"; [ $rc -eq 0 ] || exit $rc
done
N=${N:-4} bash tools/gpurun/train_ab.sh $(basename $O) "$@"
