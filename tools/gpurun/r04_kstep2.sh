#!/bin/bash
# k_step with two board pairs per lane (build/lib_env_np2.so): env GPU tests on that build, then the
# 2^26-board A/B against the product, libraries alternated over processes.
set -o pipefail
O=gpurun_out/r04_kstep2; mkdir -p $O
R48_LIB=build/lib_env_np2.so timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for L in rein48_amd/lib/librein48.so build/lib_env_np2.so; do
    timeout -k 10 120 python tools/exp_kstep_ab.py $L 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
