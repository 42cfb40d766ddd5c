#!/bin/bash
# Process-per-library A/B of k_step_n builds (tools/build_variant.sh outputs, plus an A/A copy of the
# base): the step_n parity tests on every library first, then tools/exp_stepn_ab.py with ONE library
# per process, libraries alternated over 4 rounds (the same-process tool's first-position penalty is
# out of the picture).  usage: bash tools/gpurun/stepn_proc_ab.sh OUTDIR lib.so [lib.so ...]
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for L in "$@"; do
  R48_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "step_n" > $O/pytest_$(basename $L .so).log 2>&1; rc=$?
  echo "$(basename $L): $(tail -1 $O/pytest_$(basename $L .so).log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3 4; do for L in "$@"; do
  R48_LIB=$L timeout -k 10 120 python tools/exp_stepn_ab.py $L 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
