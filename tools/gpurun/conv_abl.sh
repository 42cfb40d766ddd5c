#!/bin/bash
# GPU job: tools/exp_conv.py over the product library and variant libraries (forward and reversed
# order), then the kernel breakdown of the config-5 update (tools/gpurun/dqn_prof.sh).
# usage: bash tools/gpurun/conv_abl.sh OUT lib.so ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
P=rein48_amd/lib/librein48.so
REV=$(printf '%s\n' "$@" | tac | tr '\n' ' ')
timeout -k 10 300 python -u tools/exp_conv.py 65536 $P "$@" > $O/exp_conv.txt 2>&1 \
&& timeout -k 10 300 python -u tools/exp_conv.py 65536 $REV $P >> $O/exp_conv.txt 2>&1 && grep -v amdgpu.ids $O/exp_conv.txt \
&& { [ -n "$NOPROF" ] || bash tools/gpurun/dqn_prof.sh $O/prof; }
