#!/bin/bash
# Third scheduler batch (round 6): LLVM's AMDGPU register-pressure trackers
# (-amdgpu-use-amdgpu-trackers) on top of each file's shipped flags -- k_cnn_train (t_trk), the
# rollout megakernels (p_trk), the ResNet acting kernel (r_trk): parity tests of each variant, then
# one process per library and round against the product (t_base) and its A/A copy (t_baseAA).
# usage: bash tools/gpurun/sched_ab3.sh OUT
set -o pipefail
NAME=$1; O=gpurun_out/$1; mkdir -p $O
V=varlib
t() { R48_LIB=$1 timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q --timeout 300 --timeout-method thread -k "$3" > $O/pytest_$(basename $1 .so).log 2>&1; rc=$?; echo "$(basename $1): $(tail -1 $O/pytest_$(basename $1 .so).log)"; return $rc; }
t $V/t_trk.so tests/test_a3c_gpu.py "fused_cnn_update or per_board_weights or trainer_fused_update" && t $V/p_trk.so tests/test_a3c_gpu.py "rollout or policy" && t $V/r_trk.so tests/test_dqn_gpu.py "resnet or act or trainer" || exit 1
N=4 bash tools/gpurun/train_ab.sh $NAME/train $V/t_base.so $V/t_trk.so $V/t_baseAA.so > /dev/null || exit 1
N=4 bash tools/gpurun/rollout_proc_ab.sh $NAME/rollout $V/t_base.so $V/p_trk.so $V/t_baseAA.so > /dev/null || exit 1
for i in 1 2 3 4; do
  if [ $((i % 2)) -eq 0 ]; then L="t_baseAA r_trk t_base"; else L="t_base r_trk t_baseAA"; fi
  for l in $L; do
    echo "$l $(timeout -k 10 300 python -u tools/exp_resnet_fused.py 2097152 $V/$l.so 2>&1 | grep -v amdgpu.ids)" >> $O/resnet.txt || exit 1
  done
done
cat $O/train/timing.txt $O/rollout/timing.txt
python3 -c "
import json
for l in open('$O/resnet.txt'):
    n, js = l.split(' ', 1); d = json.loads(js)
    print('%-10s q %.3f act %.3f hash %d' % (n, d['q']['ms'], d['act']['ms'], d['q_bits_hash']))"
