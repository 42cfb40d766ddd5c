#!/bin/bash
# The max-memory-clause scheduler on the other MFMA kernels (round 6): parity tests of each variant
# library, then one-process-per-library timings against the product and its A/A copy:
# rollout megakernel (p_polmc), the MLP rollout (p_mlpmc) and update (p_mtrmc) via the config-3 MLP
# step, the ResNet act (p_resmc) via the config-5 step.
# usage: bash tools/gpurun/sched_ab.sh OUT
set -o pipefail
NAME=$1; O=gpurun_out/$1; mkdir -p $O
V=varlib
t() { R48_LIB=$1 timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q --timeout 300 --timeout-method thread -k "$3" > $O/pytest_$(basename $1 .so).log 2>&1; rc=$?; echo "$(basename $1): $(tail -1 $O/pytest_$(basename $1 .so).log)"; return $rc; }
t $V/p_polmc.so tests/test_a3c_gpu.py "rollout or policy" && t $V/p_mlpmc.so tests/test_a3c_gpu.py "mlp" && t $V/p_mtrmc.so tests/test_a3c_gpu.py "mlp" && t $V/p_resmc.so tests/test_dqn_gpu.py "resnet or act or trainer" || exit 1
N=4 bash tools/gpurun/rollout_proc_ab.sh $NAME/rollout $V/p_base.so $V/p_polmc.so $V/p_baseAA.so > /dev/null || exit 1
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 0 ]; then L="p_baseAA p_mtrmc p_mlpmc p_base"; else L="p_base p_mlpmc p_mtrmc p_baseAA"; fi
  for l in $L; do
    R48_LIB=$V/$l.so timeout -k 10 300 python -u -c "
import torch, bench
r = bench.a3c_config3(torch.device('cuda', 0), 1, 1 << 20, mode='reference', features='values', net='mlp', bf16=False)
print('$l', 'mlp rollout %.3f update %.3f ms' % (r['rollout_ms'], r['update_ms']), flush=True)" 2>&1 | grep -v amdgpu.ids >> $O/mlp.txt || exit 1
  done
done
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 0 ]; then L="p_baseAA p_resmc p_base"; else L="p_base p_resmc p_baseAA"; fi
  for l in $L; do
    R48_LIB=$V/$l.so timeout -k 10 300 python -u -c "
import torch, bench
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print('$l', 'act %.3f update %.3f ms' % (r['act_ms'], r['update_ms']), flush=True)" 2>&1 | grep -v amdgpu.ids >> $O/dqn.txt || exit 1
  done
done
cat $O/rollout/timing.txt $O/mlp.txt $O/dqn.txt
