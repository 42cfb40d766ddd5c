#!/bin/bash
# GPU job: A/B timing of k_cnn_train variant libraries against the product (tools/exp_train.py,
# interleaved, gradient digests compared), then per-phase stamps of stamped builds
# (tools/stamp_train.py).  usage: bash tools/gpurun/train_var.sh "<variant.so ...>" "<stamp.so ...>"
set -o pipefail
O=gpurun_out/train_var; mkdir -p $O
P=rein48_amd/lib/librein48.so
timeout -k 10 400 python -u tools/exp_train.py 16777216 $P $1 $P $1 > $O/train.txt 2>&1 && cat $O/train.txt || exit 1
for s in $2; do
    timeout -k 10 120 python -u tools/exp_train_stamps.py $s > $O/stamps_$(basename $s .so).txt 2>&1 && cat $O/stamps_$(basename $s .so).txt || exit 1
done
