#!/bin/bash
# Config-5 update timing with the BN applies folded into the next conv's operand load
# (ResNetTrainStep fold_bn=True) vs the separate apply passes (default), one process per arm,
# alternated. usage: N=4 bash tools/gpurun/dqn_fold_ab.sh OUT
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for i in $(seq ${N:-4}); do
  if [ $((i % 2)) -eq 0 ]; then ARMS="fold apply"; else ARMS="apply fold"; fi
  for a in $ARMS; do
    timeout -k 10 300 python -u -c "
import torch, bench
from rein48_amd.dqn import train_step as T
if '$a' == 'fold':
    f = T.ResNetTrainStep.__init__
    T.ResNetTrainStep.__init__ = lambda self, net, fold_bn=True: f(self, net, fold_bn=True)
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print('$a', 'act %.2f ms update %.2f ms' % (r['act_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
  done
done
cat $O/timing.txt
