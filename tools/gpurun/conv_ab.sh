#!/bin/bash
# GPU job: conv parity tests, then A/B timings (tools/exp_conv.py, inputs rotated past the Infinity
# Cache) of the product library against variant libraries.  usage: bash tools/gpurun/conv_ab.sh <lib.so> ...
set -o pipefail
O=gpurun_out/conv_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dqn_gpu.py -k "conv or head or train_step or pack" > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] \
&& timeout -k 10 300 python -u tools/exp_conv.py 65536 rein48_amd/lib/librein48.so "$@" rein48_amd/lib/librein48.so > $O/ab.txt 2>&1; cat $O/ab.txt
