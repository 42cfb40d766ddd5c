#!/bin/bash
# GPU job: conv parity tests, timings of the product and ablation libraries (tools/conv_variants.py),
# wgrad phase stamps (tools/stamp_conv.py)
set -o pipefail
O=gpurun_out/abl; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dqn_gpu.py -k "conv or onehot or head" > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] \
&& timeout -k 10 120 python -u tools/exp_conv_stamps.py build/lib_conv_stamp.so > $O/stamps.txt 2>&1; cat $O/stamps.txt \
&& timeout -k 10 300 python -u tools/exp_conv.py 65536 rein48_amd/lib/librein48.so "$@" > $O/abl.txt 2>&1; cat $O/abl.txt
