#!/bin/bash
# GPU job: DQN GPU tests on a conv variant (installed over the product library in this box's copy),
# conv timings product vs variant, and the variant's wgrad stamps.  usage: bash tools/gpurun/conv_ds.sh <variant.so> [stamp.so]
set -o pipefail
O=gpurun_out/conv_ds; mkdir -p $O
timeout -k 10 300 python -u tools/exp_conv.py 65536 rein48_amd/lib/librein48.so $1 rein48_amd/lib/librein48.so $1 > $O/conv.txt 2>&1 && cat $O/conv.txt || exit 1
if [ -n "$2" ]; then timeout -k 10 120 python tools/exp_conv_stamps.py $2 > $O/stamps.txt 2>&1 && cat $O/stamps.txt || exit 1; fi
cp $1 rein48_amd/lib/librein48.so && timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py > $O/pytest.txt 2>&1; tail -2 $O/pytest.txt
