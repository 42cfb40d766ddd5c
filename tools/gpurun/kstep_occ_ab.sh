#!/bin/bash
# k_step at 2^26 boards with its occupancy limited by dynamic LDS per workgroup (40 / 27 / 20 KB:
# 4 / 6 / 8 waves per SIMD... of the 8 the shipped grid allows), vs the product; processes alternated.
set -o pipefail
O=gpurun_out/kstep_occ; mkdir -p $O
for i in 1 2; do for L in rein48_amd/lib/librein48.so build/lib_env_lds40960.so build/lib_env_lds27648.so build/lib_env_lds20480.so; do
  timeout -k 10 120 python tools/exp_kstep_ab.py $L 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
