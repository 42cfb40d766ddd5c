#!/bin/bash
# GPU job: config-5 conv parity tests, A/B of the conv kernels against variant libraries, then the
# kernel breakdown of one update (tools/prof_dqn.py).  usage: bash tools/gpurun/conv.sh <variant.so> ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/conv; mkdir -p $O
P=rein48_amd/lib/librein48.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dqn_gpu.py -k "conv or onehot or head" > $O/pytest_conv.txt 2>&1; rc=$?; tail -8 $O/pytest_conv.txt; [ $rc -eq 0 ] \
&& timeout -k 10 200 python -u tools/exp_conv.py 65536 $P "$@" > $O/exp_conv.txt 2>&1 && cat $O/exp_conv.txt \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o dqn -- python3 tools/prof_dqn.py > $O/prof_dqn.log 2>&1 && tail -2 $O/prof_dqn.log
