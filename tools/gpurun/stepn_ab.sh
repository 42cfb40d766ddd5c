#!/bin/bash
# A/B of k_step_n library variants (varlib/*.so built by tools/build_variant.sh) at 2^20 boards,
# K = 20 and K = 1000, with a bit-level digest per library.  usage: bash tools/gpurun/stepn_ab.sh lib.so ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/exp_stepn_ab.py "$@" 2>&1 | tee gpurun_out/stepn_ab.txt
