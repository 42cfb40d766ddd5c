#!/bin/bash
# k_step (one step per launch, boards through HBM) at 2^26 boards: the env GPU tests on the second
# library given (the variant), then tools/exp_kstep_ab.py for every library, alternated, 3 rounds.
# usage: bash tools/gpurun/kstep_ab.sh OUTDIR rein48_amd/lib/librein48.so build/lib_variant.so [...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
R48_LIB=${2:-$1} timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for L in "$@"; do
  timeout -k 10 120 python tools/exp_kstep_ab.py $L 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
