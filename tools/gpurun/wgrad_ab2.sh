#!/bin/bash
# k_conv_wgrad, one wave per SIMD with the fragment reads pipelined kAhead pairs ahead (round 6):
# the DQN GPU tests on the product library, then one process per library and round (order rotated)
# of tools/exp_conv.py's wgrad cases: product (4 waves, 6 ahead), q_prev (the committed 8-wave
# split-K kernel), 7 and 3 ahead, q_newAA (a byte copy of the product: the A/A control); then the
# config-5 act + update for product / q_prev / q_newAA.  usage: bash tools/gpurun/wgrad_ab2.sh OUT
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
V=varlib
P=rein48_amd/lib/librein48.so
timeout -k 10 600 python -u -m pytest tests/test_dqn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dqn.log 2>&1; rc=$?; tail -2 $O/pytest_dqn.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  case $i in 1) L="$P $V/q_prev.so $V/wg_w4a7.so $V/wg_w4a3.so $V/q_newAA.so";;
             2) L="$V/q_newAA.so $V/wg_w4a3.so $V/wg_w4a7.so $V/q_prev.so $P";;
             3) L="$V/q_prev.so $P $V/q_newAA.so $V/wg_w4a7.so $V/wg_w4a3.so";; esac
  for l in $L; do
    CASES=wgrad64,wgrad32 timeout -k 10 300 python -u tools/exp_conv.py 65536 $l 2>&1 | grep -v amdgpu.ids >> $O/exp_conv.txt || exit 1
  done
done
cat $O/exp_conv.txt
for i in 1 2 3; do
  if [ $((i % 2)) -eq 0 ]; then L="q_newAA q_prev new"; else L="new q_prev q_newAA"; fi
  for l in $L; do
    if [ $l = new ]; then LIB=$P; else LIB=$V/$l.so; fi
    R48_LIB=$LIB timeout -k 10 300 python -u -c "
import torch, bench
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print('$l', 'act %.3f update %.3f ms' % (r['act_ms'], r['update_ms']), flush=True)" 2>&1 | grep -v amdgpu.ids >> $O/dqn.txt || exit 1
  done
done
cat $O/dqn.txt
