#!/bin/bash
# Config-5 act/update timing with the bench's update(sync=False) vs a forced update(sync=True)
# (the loss read back to the host inside every update), one process per arm, alternated.
# usage: N=4 bash tools/gpurun/dqn_sync_ab.sh OUT
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for i in $(seq ${N:-4}); do
  if [ $((i % 2)) -eq 0 ]; then ARMS="async sync"; else ARMS="sync async"; fi
  for a in $ARMS; do
    timeout -k 10 300 python -u -c "
import torch, bench
from rein48_amd.dqn.trainer import DQNTrainer
if '$a' == 'sync':
    f = DQNTrainer.update
    DQNTrainer.update = lambda self, batch=None, sync=True: f(self, batch, True)
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print('$a', 'act %.2f ms update %.2f ms' % (r['act_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
  done
done
cat $O/timing.txt
