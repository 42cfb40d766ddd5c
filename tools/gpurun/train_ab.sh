#!/bin/bash
# GPU job: fused A3C update parity tests, then A/B timing of the product library against variant
# libraries (tools/build_variant.sh) and the per-phase stamps (tools/stamp_train.py).
# usage: bash tools/gpurun/train_ab.sh <variant.so> ...
set -o pipefail
O=gpurun_out/train_ab; mkdir -p $O
P=rein48_amd/lib/librein48.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_a3c_gpu.py \
    -k "update or trainer" > $O/pytest.txt 2>&1 && tail -2 $O/pytest.txt \
&& timeout -k 10 300 python -u tools/exp_train.py 16777216 $P "$@" $P "$@" > $O/train.txt 2>&1 && cat $O/train.txt \
&& if [ -f build/lib_train_stamp.so ]; then timeout -k 10 120 python -u tools/exp_train_stamps.py build/lib_train_stamp.so > $O/stamps.txt 2>&1 && cat $O/stamps.txt; fi
