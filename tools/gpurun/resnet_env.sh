#!/bin/bash
# Fused ResNet-10 inference timing at 2^21 boards (tools/exp_resnet_fused.py), then the env
# profiles (prof_env.sh).  usage: bash tools/gpurun/resnet_env.sh r03
set -o pipefail
R=${1:-r03}
mkdir -p gpurun_out/resnet
timeout -k 10 200 python tools/exp_resnet_fused.py > gpurun_out/resnet/exp_resnet_fused.txt 2>&1 && cat gpurun_out/resnet/exp_resnet_fused.txt \
&& bash tools/gpurun/prof_env.sh $R
