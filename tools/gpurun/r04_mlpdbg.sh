#!/bin/bash
# MLP update gradient diagnostic (row counts across tiles-per-wave), then the remaining A3C tests/timings.
set -o pipefail
O=gpurun_out/r04_mlp; mkdir -p $O
timeout -k 10 300 python -u tools/exp_mlp_grad_debug.py > $O/grad_debug.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/grad_debug.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/exp_learning.py gpurun_out/r04_learn/learning.json --a3c-updates 2000 --dqn-steps 3000 > gpurun_out/r04_learn.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04_learn.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_learning_gpu.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04_learn_pytest.log 2>&1; tail -6 gpurun_out/r04_learn_pytest.log
