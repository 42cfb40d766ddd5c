#!/bin/bash
# Second scheduler batch (round 6): parity tests of each variant, then one-process-per-library
# timings against the product and its A/A copy: rollout (iterative-ilp instead of max-ilp), ResNet act
# (max-ilp), k_cnn_train (max-memory-clause + no unclustered high-RP reschedule).
# usage: bash tools/gpurun/sched_ab2.sh OUT
set -o pipefail
NAME=$1; O=gpurun_out/$1; mkdir -p $O
V=varlib
t() { R48_LIB=$1 timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q --timeout 300 --timeout-method thread -k "$3" > $O/pytest_$(basename $1 .so).log 2>&1; rc=$?; echo "$(basename $1): $(tail -1 $O/pytest_$(basename $1 .so).log)"; return $rc; }
t $V/q_politilp.so tests/test_a3c_gpu.py "rollout or policy" && t $V/q_resmaxilp.so tests/test_dqn_gpu.py "resnet or act or trainer" && t $V/q_trnohrp.so tests/test_a3c_gpu.py "fused_cnn_update or per_board_weights or trainer_fused_update" || exit 1
N=4 bash tools/gpurun/rollout_proc_ab.sh $NAME/rollout $V/q_base.so $V/q_politilp.so $V/q_baseAA.so > /dev/null || exit 1
N=4 bash tools/gpurun/train_ab.sh $NAME/train $V/q_base.so $V/q_trnohrp.so $V/q_baseAA.so > /dev/null || exit 1
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 0 ]; then L="q_baseAA q_resmaxilp q_base"; else L="q_base q_resmaxilp q_baseAA"; fi
  for l in $L; do
    R48_LIB=$V/$l.so timeout -k 10 300 python -u -c "
import torch, bench
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print('$l', 'act %.3f update %.3f ms' % (r['act_ms'], r['update_ms']), flush=True)" 2>&1 | grep -v amdgpu.ids >> $O/dqn.txt || exit 1
  done
done
cat $O/rollout/timing.txt $O/train/timing.txt $O/dqn.txt
