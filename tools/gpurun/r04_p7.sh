#!/bin/bash
# Draw contract 3 (Philox4x32-7 step draws): env + A3C + learning GPU tests, then the K = 20 / 1000 timing.
set -o pipefail
O=gpurun_out/r04_p7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_env_gpu.py tests/test_a3c_gpu.py tests/test_learning_gpu.py tests/test_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python tools/exp_stepn_ab.py 2>&1 | grep -v amdgpu.ids > $O/ab_product.txt; rc=$?; cat $O/ab_product.txt; exit $rc
