#!/bin/bash
# Config-5 act/update timing of two ResNetTrainStep settings, one process per arm, alternated:
# arm "default" vs arm KNOB (a keyword of ResNetTrainStep.__init__ forced to VALUE).
# usage: N=4 bash tools/gpurun/dqn_knob_ab.sh OUT KNOB VALUE     e.g. overlap False, fold_bn True
set -o pipefail
O=gpurun_out/$1; K=$2; V=$3; mkdir -p $O
for i in $(seq ${N:-4}); do
  if [ $((i % 2)) -eq 0 ]; then ARMS="$K=$V default"; else ARMS="default $K=$V"; fi
  for a in $ARMS; do
    timeout -k 10 300 python -u -c "
import torch, bench
from rein48_amd.dqn import train_step as T
if '$a' != 'default':
    f = T.ResNetTrainStep.__init__
    def init(self, net, **kw):
        kw['$K'] = $V
        f(self, net, **kw)
    T.ResNetTrainStep.__init__ = init
r = bench.dqn_config5(torch.device('cuda', 0), 0x20485EED, 1 << 21)
print('$a', 'act %.2f ms update %.2f ms' % (r['act_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids >> $O/timing.txt || exit 1
  done
done
cat $O/timing.txt
