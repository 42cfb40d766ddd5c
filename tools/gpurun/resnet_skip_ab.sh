#!/bin/bash
# k_resnet_q skip connection on the VALU instead of an identity MFMA (round 6): the DQN GPU tests on
# the product library, then one process per library and round (alternated order) of
# tools/exp_resnet_fused.py (Q-only and acting at 2^21 boards, with a bit hash of Q) and of the
# config-5 act + update: product vs q_prev (identity MFMA) vs q_newAA (a byte copy of the product).
# usage: bash tools/gpurun/resnet_skip_ab.sh OUT
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
V=varlib
P=rein48_amd/lib/librein48.so
timeout -k 10 600 python -u -m pytest tests/test_dqn_gpu.py tests/test_dqn.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dqn.log 2>&1; rc=$?; tail -2 $O/pytest_dqn.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 0 ]; then L="$V/q_newAA.so $V/q_prev.so $P"; else L="$P $V/q_prev.so $V/q_newAA.so"; fi
  for l in $L; do
    echo "$(basename $l) $(timeout -k 10 300 python -u tools/exp_resnet_fused.py 2097152 $l 2>&1 | grep -v amdgpu.ids)" >> $O/fused.txt || exit 1
  done
done
cat $O/fused.txt
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
