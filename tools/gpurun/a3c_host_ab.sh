#!/bin/bash
# A/B of the A3C host path: config-3 train-step timings (bench.a3c_config3, CNN textbook / reference and
# the reference MLP) of this tree vs an older tree exported to build/ab/oldrepo (same librein48.so),
# alternated over N rounds, after the A3C GPU tests of this tree.  usage: N=3 bash tools/gpurun/a3c_host_ab.sh OUT
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_a3c_gpu.py tests/test_checkpoint_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${N:-2}); do for T in . build/ab/oldrepo; do
(cd $T && timeout -k 10 300 python -u -c "
import torch, bench
d = torch.device('cuda', 0)
for name, kw in (('cnn textbook', dict(mode='textbook', features='exponents')), ('cnn reference', dict(mode='reference', features='values')),
                 ('mlp reference', dict(mode='reference', features='values', net='mlp', bf16=False))):
    r = bench.a3c_config3(d, 0x20485EED, 1 << 20, **kw)
    print('$T', name, 'rollout %.2f ms update %.2f ms' % (r['rollout_ms'], r['update_ms']), flush=True)
" 2>&1 | grep -v amdgpu.ids) >> $O/timing.txt || exit 1
done; done
cat $O/timing.txt
