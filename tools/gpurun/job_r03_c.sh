#!/bin/bash
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py > $O/pytest_dqn.txt 2>&1; tail -15 $O/pytest_dqn.txt
bash tools/gpurun/train_ab.sh build/lib_train_head.so
